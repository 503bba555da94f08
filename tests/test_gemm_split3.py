"""fp32-accurate split GEMMs (NTS_GEMM_SPLIT3, csrc/gemm3.hip) vs fp64 and vs
the fp32-input MFMA path.

Bar: on every shape and fused variant the layer GEMMs take (NN with the
relu/dropout epilogue, row-gathered NN, TN with the relu/dropout backward,
row-gathered TN) the split path's error against an fp64 GEMM of the same fp32
operands is at most 1.25x the fp32 MFMA path's error (plus 1e-7 of the
operand scale), i.e. the same precision class as the reference's fp32 GEMM;
the dropout keep mask is the fp32 path's; results are deterministic.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def ctxs():
    from nts import _abi
    from nts.hip import HipContext
    f32 = HipContext(0, seed=2000)
    s3 = HipContext(0, seed=2000)
    s3.set_gemm_mode(_abi.NTS_GEMM_SPLIT3_ALL)  # every shape on the split kernels
    return f32, s3


def _errs(got_f32, got_s3, ref, scale):
    """max |err| / scale (scale = |A| |B| per element) of each path"""
    e32 = ((got_f32.double() - ref).abs() / scale).max().item()
    es3 = ((got_s3.double() - ref).abs() / scale).max().item()
    return e32, es3


def _check(e32, es3):
    assert es3 <= 1.25 * e32 + 1e-7, (es3, e32)
    assert es3 < 5e-7, es3


def _padded(rows, cols, g, pad=32):
    ld = (cols + 31) // 32 * 32 + pad
    big = torch.full((rows, ld), float("nan"), device=DEV)
    A = big[:, :cols]
    A.copy_(torch.randn(rows, cols, device=DEV, generator=g))
    return A


@pytest.mark.parametrize("M,N,K", [(136076, 128, 602), (4099, 256, 301), (2100, 64, 602),
                                   (700, 128, 3), (257, 128, 100), (5000, 192, 33), (300, 16, 64)])
def test_split3_gemm_nn(ctxs, M, N, K):
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(M + 3 * N + K)
    A = _padded(M, K, g)
    B = torch.randn(K, N, device=DEV, generator=g) + torch.arange(N, device=DEV) * 0.01
    C32 = torch.full((M, N), float("nan"), device=DEV)
    C3 = torch.full((M, N), float("nan"), device=DEV)
    f32.gemm(A, B, C32)
    s3.gemm(A, B, C3)
    ref = A.double() @ B.double()
    scale = A.double().abs() @ B.double().abs() + 1e-30
    torch.cuda.synchronize()
    assert not torch.isnan(C3).any()
    _check(*_errs(C32, C3, ref, scale))
    C3b = torch.empty_like(C3)
    s3.gemm(A, B, C3b)
    torch.cuda.synchronize()
    assert torch.equal(C3, C3b)


@pytest.mark.parametrize("M,N,K", [(602, 128, 135758), (602, 128, 20000), (100, 256, 3000),
                                   (256, 256, 999), (333, 128, 777), (41, 64, 300)])
def test_split3_gemm_tn(ctxs, M, N, K):
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(M * 5 + N + K)
    A = _padded(K, M, g)
    B = torch.randn(K, N, device=DEV, generator=g)
    C32 = torch.full((M, N), float("nan"), device=DEV)
    C3 = torch.full((M, N), float("nan"), device=DEV)
    f32.gemm(A, B, C32, trans_a=True)
    s3.gemm(A, B, C3, trans_a=True)
    ref = A.double().t() @ B.double()
    scale = A.double().abs().t() @ B.double().abs() + 1e-30
    torch.cuda.synchronize()
    assert not torch.isnan(C3).any()
    _check(*_errs(C32, C3, ref, scale))
    C3b = torch.empty_like(C3)
    s3.gemm(A, B, C3b, trans_a=True)
    torch.cuda.synchronize()
    assert torch.equal(C3, C3b)


@pytest.mark.parametrize("M,N,K,p", [(136076, 128, 602, 0.5), (4001, 256, 128, 0.5),
                                     (1000, 128, 128, 0.0), (2050, 64, 77, 0.2)])
def test_split3_relu_dropout_epilogue(ctxs, M, N, K, p):
    """Same keep mask as the fp32 path (the documented Philox stream), values
    within the split path's precision."""
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(M + N + K + 1)
    A = torch.randn(M, K, device=DEV, generator=g)
    B = torch.randn(K, N, device=DEV, generator=g)
    C32 = torch.empty(M, N, device=DEV)
    C3 = torch.empty(M, N, device=DEV)
    seed, offset = 0x1234_5678_9ABC, 77
    f32.gemm_relu_dropout(A, B, C32, p=p, seed=seed, offset=offset)
    s3.gemm_relu_dropout(A, B, C3, p=p, seed=seed, offset=offset)
    Z = A.double() @ B.double()
    scale = A.double().abs() @ B.double().abs() + 1e-30
    torch.cuda.synchronize()
    clear = Z.abs() > 1e-5 * scale  # relu decisions away from rounding of 0
    assert torch.equal((C32 != 0) & clear, (C3 != 0) & clear)
    s = 1.0 / (1.0 - p)
    ref = torch.where(C32 != 0, torch.relu(Z) * s, torch.zeros_like(Z))
    e32 = ((C32.double() - ref).abs() / (scale * s))[clear].max().item()
    es3 = ((C3.double() - ref).abs() / (scale * s))[clear].max().item()
    _check(e32, es3)


@pytest.mark.parametrize("M,N,K", [(602, 128, 135758), (602, 128, 5000), (1000, 256, 999)])
def test_split3_gemm_tn_masked(ctxs, M, N, K):
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(M * 3 + N + K)
    A = torch.randn(K, M, device=DEV, generator=g)
    G = torch.randn(K, N, device=DEV, generator=g)
    X = torch.relu(torch.randn(K, N, device=DEV, generator=g))
    C32 = torch.empty(M, N, device=DEV)
    C3 = torch.empty(M, N, device=DEV)
    f32.gemm_tn_masked(A, G, X, C32, scale=2.0)
    s3.gemm_tn_masked(A, G, X, C3, scale=2.0)
    Bm = G.double() * (X > 0).double() * 2.0
    ref = A.double().t() @ Bm
    scale = A.double().abs().t() @ Bm.abs() + 1e-30
    torch.cuda.synchronize()
    _check(*_errs(C32, C3, ref, scale))


@pytest.mark.parametrize("M,N,K", [(228656, 128, 602), (3000, 128, 602), (2500, 256, 100)])
def test_split3_gemm_gather_rows(ctxs, M, N, K):
    """Transform-first bottom layer: C = table[rows] W with rows gathered in
    the GEMM == the split GEMM of the gathered copy, bit for bit."""
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(M + K + 5)
    V = M + M // 3 + 11
    table = _padded(V, K, g)
    rows = torch.randperm(V, device=DEV, generator=g)[:M].to(torch.int32)
    W = torch.randn(K, N, device=DEV, generator=g)
    C32 = torch.empty(M, N, device=DEV)
    C3 = torch.empty(M, N, device=DEV)
    f32.gemm_gather(table, rows, W, C32)
    s3.gemm_gather(table, rows, W, C3)
    Xg = torch.empty(M, (K + 31) // 32 * 32, device=DEV)[:, :K]  # 16-byte aligned rows
    Xg.copy_(table[rows.long()])
    C3c = torch.empty(M, N, device=DEV)
    s3.gemm(Xg, W, C3c)
    ref = Xg.double() @ W.double()
    scale = Xg.double().abs() @ W.double().abs() + 1e-30
    torch.cuda.synchronize()
    assert torch.equal(C3, C3c)
    _check(*_errs(C32, C3, ref, scale))


@pytest.mark.parametrize("M,N,K", [(602, 128, 228656), (602, 128, 5000), (100, 256, 3000)])
def test_split3_gemm_tn_gather_rows(ctxs, M, N, K):
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(M * N + K + 9)
    V = K + K // 2 + 5
    table = _padded(V, M, g)
    rows = torch.randint(0, V, (K,), device=DEV, generator=g).to(torch.int32)
    G = torch.randn(K, N, device=DEV, generator=g)
    C32 = torch.empty(M, N, device=DEV)
    C3 = torch.empty(M, N, device=DEV)
    f32.gemm_tn_gather(table, rows, G, C32)
    s3.gemm_tn_gather(table, rows, G, C3)
    Xg = table[rows.long()].contiguous()
    ref = Xg.double().t() @ G.double()
    scale = Xg.double().abs().t() @ G.double().abs() + 1e-30
    torch.cuda.synchronize()
    _check(*_errs(C32, C3, ref, scale))


def test_split3_error_distribution_report(ctxs):
    """The headline shape (C2 bottom layer, 136,076 x 602 x 128): mean and max
    normalised error of both paths, printed for DESIGN.md, and the split path
    not worse on average."""
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(42)
    A = torch.rand(136076, 608, device=DEV, generator=g)[:, :602]  # the padded pitch; non-negative
    B = torch.randn(602, 128, device=DEV, generator=g) * 0.05
    C32 = torch.empty(136076, 128, device=DEV)
    C3 = torch.empty_like(C32)
    f32.gemm(A, B, C32)
    s3.gemm(A, B, C3)
    ref = A.double() @ B.double()
    scale = A.double().abs() @ B.double().abs() + 1e-30
    torch.cuda.synchronize()
    r32 = (C32.double() - ref).abs() / scale
    r3 = (C3.double() - ref).abs() / scale
    print(f"\n[split3] fp32 MFMA: mean {r32.mean().item():.3e} max {r32.max().item():.3e}; "
          f"split3: mean {r3.mean().item():.3e} max {r3.max().item():.3e}")
    assert r3.mean().item() <= 1.1 * r32.mean().item()
    _check(r32.max().item(), r3.max().item())
