"""fp32-exact row-gathered GEMMs over whole feature rows (csrc/gemmx3.hip):
the transform-first bottom layer's H = X[src] W and dW = X[src]^T dH in the
headline's arithmetic (every fp32 operand split exactly into three bf16
pieces in the kernel, six products, fp32 accumulate).

Bar (as tests/test_gemm_split3.py): error against an fp64 GEMM of the same
fp32 operands at most 1.25x the fp32-input MFMA path's (plus 1e-7 of the
operand scale) on every shape the kernels take — the reference's fp32
`x.matmul(W)` precision class (core/NtsScheduler.hpp:859-862); NaN in the
table's pad columns never reaches a stored element; deterministic.
"""
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
    s3.set_gemm_mode(_abi.NTS_GEMM_SPLIT3)
    return f32, s3


def _table(V, K, g, pitch=None):
    """[V, K] view of a table whose pad columns hold NaN (row pitch: 640 floats
    for K = 602, the padded feature table's)"""
    ld = pitch or ((K + 31) // 32 * 32 + 32)
    big = torch.full((V, ld), float("nan"), device=DEV)
    big[:, :K] = torch.randn(V, K, device=DEV, generator=g)
    return big[:, :K]


def _check(got32, got3, ref, scale):
    e32 = ((got32.double() - ref).abs() / scale).max().item()
    e3 = ((got3.double() - ref).abs() / scale).max().item()
    assert e3 <= 1.25 * e32 + 1e-7, (e3, e32)
    assert e3 < 5e-7, e3


@pytest.mark.parametrize("M,N,K", [(602, 128, 228656), (602, 128, 4099), (640, 128, 3001),
                                   (100, 256, 3000), (128, 128, 70001), (41, 128, 300),
                                   (602, 128, 257)])
def test_x3_tn_gather(ctxs, M, N, K):
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + K)
    V = K + K // 2 + 5
    table = _table(V, M, g)
    rows = torch.randint(0, V, (K,), device=DEV, generator=g).to(torch.int32)
    rows, _ = torch.sort(rows)  # the sampler's src lists are ascending
    G = torch.randn(K, N, device=DEV, generator=g) * torch.rand(K, 1, device=DEV, generator=g)
    C32 = torch.empty(M, N, device=DEV)
    C3 = torch.full((M, N), float("nan"), device=DEV)
    f32.gemm_tn_gather(table, rows, G, C32)
    s3.gemm_tn_gather(table, rows, G, C3)
    Xg = table[rows.long()].double()
    ref = Xg.t() @ G.double()
    scale = Xg.abs().t() @ G.double().abs() + 1e-30
    torch.cuda.synchronize()
    assert not torch.isnan(C3).any()
    _check(C32, C3, ref, scale)
    C3b = torch.empty_like(C3)
    s3.gemm_tn_gather(table, rows, G, C3b)
    torch.cuda.synchronize()
    assert torch.equal(C3, C3b)


def test_x3_tn_wide_range(ctxs):
    """rows spanning many decades and tiny gradients: exact three-piece inputs
    keep every element's relative precision (no per-row scale)"""
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(11)
    M, N, K = 602, 128, 20000
    V = 30000
    table = _table(V, M, g)
    with torch.no_grad():
        table.mul_(torch.pow(10.0, torch.randint(-12, 12, (V, M), device=DEV, generator=g).float()))
    rows = torch.sort(torch.randperm(V, device=DEV, generator=g)[:K])[0].to(torch.int32)
    G = torch.randn(K, N, device=DEV, generator=g) * 1e-7
    C32 = torch.empty(M, N, device=DEV)
    C3 = torch.empty(M, N, device=DEV)
    f32.gemm_tn_gather(table, rows, G, C32)
    s3.gemm_tn_gather(table, rows, G, C3)
    Xg = table[rows.long()].double()
    ref = Xg.t() @ G.double()
    scale = Xg.abs().t() @ G.double().abs() + 1e-300
    torch.cuda.synchronize()
    _check(C32, C3, ref, scale)


@pytest.mark.parametrize("M,N,K,V", [(228656, 128, 602, 232965), (7 * 16 * 1024 * 3 + 37, 128, 602, 400000),
                                     (257, 128, 602, 300), (5000, 64, 602, 6000), (2500, 256, 100, 4000),
                                     (4000, 128, 97, 4100), (1000, 48, 129, 1200)])
def test_x3_nn_gather_bitexact(ctxs, M, N, K, V):
    """k_x3_nn7 (4-wave blocks, 7 row tiles a wave, A straight to registers,
    rounds chained; the default for the un-fused gathered NN): the gathered
    product equals the split GEMM of the gathered copy bit for bit (same
    pieces, same piece and k order), over tile counts that leave the last
    round short, several rounds, N below / above one 128-column block, K
    with a pad step; NaN in the table's pad columns never reaches an output."""
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(M + 3 * K + N)
    table = _table(V, K, g)
    rows = torch.randint(0, V, (M,), device=DEV, generator=g).to(torch.int32)
    rows, _ = torch.sort(rows)
    W = torch.randn(K, N, device=DEV, generator=g)
    C3 = torch.full((M, N), float("nan"), device=DEV)
    s3.gemm_gather(table, rows, W, C3)
    Xg = torch.empty(M, (K + 31) // 32 * 32, device=DEV)[:, :K]
    Xg.copy_(table[rows.long()])
    C3c = torch.empty(M, N, device=DEV)
    s3.gemm(Xg, W, C3c)
    torch.cuda.synchronize()
    assert not torch.isnan(C3).any()
    assert torch.equal(C3, C3c)
    if M <= 300000:
        C32 = torch.empty(M, N, device=DEV)
        f32.gemm_gather(table, rows, W, C32)
        ref = Xg.double() @ W.double()
        scale = Xg.double().abs() @ W.double().abs() + 1e-30
        torch.cuda.synchronize()
        _check(C32, C3, ref, scale)


@pytest.mark.parametrize("M,N,K,p", [(140000, 256, 100, 0.5), (60000, 128, 602, 0.3),
                                     (40000, 256, 128, 0.0)])
def test_x3_nn7_relu_dropout_dense(ctxs, M, N, K, p):
    """k_x3_nn7's relu/dropout epilogue on dense rows (reached under
    NTS_GEMM_SPLIT3_ALL when the row pitch covers whole k-steps; the default
    split mode keeps the narrow aggregate-first layers of C3 / C4 on the fp32
    MFMA kernels, which measured faster): bit-identical to
    k_gemm3_nn<relu/dropout> on the same rows at a pitch k_x3_nn7 does not take
    (same pieces, piece and k order, accumulator layout and Philox keep mask),
    and within the split path's bound of an fp64 product."""
    from nts import _abi
    from nts.hip import HipContext
    f32, s3 = ctxs
    s3all = HipContext(0, seed=2000)
    s3all.set_gemm_mode(_abi.NTS_GEMM_SPLIT3_ALL)
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    Kp = (K + 31) // 32 * 32
    Apad = torch.full((M, Kp + 32), float("nan"), device=DEV)[:, :K]  # k_x3_nn7's pitch
    Apad.copy_(torch.randn(M, K, device=DEV, generator=g))
    A4 = torch.empty(M, (K + 3) // 4 * 4 + (4 if K % 32 == 0 else 0), device=DEV)[:, :K]
    A4.copy_(Apad)  # a 16-byte pitch below Kp: k_gemm3_nn
    B = torch.randn(K, N, device=DEV, generator=g)
    seed, offset = 0x1234_5678_9ABC, 77
    C7 = torch.full((M, N), float("nan"), device=DEV)
    Cr = torch.empty(M, N, device=DEV)
    C32 = torch.empty(M, N, device=DEV)
    s3all.gemm_relu_dropout(Apad, B, C7, p=p, seed=seed, offset=offset)
    s3all.gemm_relu_dropout(A4, B, Cr, p=p, seed=seed, offset=offset)
    f32.gemm_relu_dropout(A4, B, C32, p=p, seed=seed, offset=offset)
    torch.cuda.synchronize()
    assert not torch.isnan(C7).any()
    assert torch.equal(C7, Cr)
    Z = Apad.double() @ B.double()
    scale = Apad.double().abs() @ B.double().abs() + 1e-30
    clear = Z.abs() > 1e-5 * scale
    assert torch.equal((C32 != 0) & clear, (C7 != 0) & clear)
    s = 1.0 / (1.0 - p)
    ref = torch.where(C32 != 0, torch.relu(Z) * s, torch.zeros_like(Z))
    e32 = ((C32.double() - ref).abs() / (scale * s))[clear].max().item()
    e7 = ((C7.double() - ref).abs() / (scale * s))[clear].max().item()
    assert e7 <= 1.25 * e32 + 1e-7, (e7, e32)


@pytest.mark.parametrize("M,N,K,pitch,p", [(140390, 256, 100, 100, 0.5), (20000, 128, 128, 128, 0.3),
                                           (9000, 48, 37, 40, 0.0)])
def test_x3_nnk_short_reduction(ctxs, M, N, K, pitch, p):
    """k_x3_nnk (round 6: dense rows, K <= 128, the whole W image in LDS; the
    default for C3 / C4's aggregate-first bottom layer): every row
    bit-identical to k_gemm3_nn's on the same rows (its first 4,000, below
    k_x3_nnk's 4,096-row floor: same pieces, products, k order and keep mask),
    and within the split path's bound of an fp64 product."""
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.empty(M, pitch, device=DEV)[:, :K]
    A.copy_(torch.randn(M, K, device=DEV, generator=g))
    B = torch.randn(K, N, device=DEV, generator=g)
    seed, offset = 0x0DDB_1A5E_5BAD_5EED, 5
    Ck = torch.full((M, N), float("nan"), device=DEV)
    C32 = torch.empty(M, N, device=DEV)
    s3.gemm_relu_dropout(A, B, Ck, p=p, seed=seed, offset=offset)
    f32.gemm_relu_dropout(A, B, C32, p=p, seed=seed, offset=offset)
    from nts import _abi
    from nts.hip import HipContext
    s3all = HipContext(0, seed=2000)
    s3all.set_gemm_mode(_abi.NTS_GEMM_SPLIT3_ALL)
    m = 4000
    Cg = torch.empty(m, N, device=DEV)
    s3all.gemm_relu_dropout(A[:m], B, Cg, p=p, seed=seed, offset=offset)
    torch.cuda.synchronize()
    assert not torch.isnan(Ck).any()
    assert torch.equal(Ck[:m], Cg)
    Z = A.double() @ B.double()
    scale = A.double().abs() @ B.double().abs() + 1e-30
    clear = Z.abs() > 1e-5 * scale
    assert torch.equal((C32 != 0) & clear, (Ck != 0) & clear)
    s = 1.0 / (1.0 - p)
    ref = torch.where(C32 != 0, torch.relu(Z) * s, torch.zeros_like(Z))
    e32 = ((C32.double() - ref).abs() / (scale * s))[clear].max().item()
    ek = ((Ck.double() - ref).abs() / (scale * s))[clear].max().item()
    assert ek <= 1.25 * e32 + 1e-7, (ek, e32)


@pytest.mark.parametrize("K,M,N,pitch", [(140390, 100, 256, 128), (30000, 64, 128, 64),
                                         (5000, 100, 128, 104)])
def test_x3_tn_masked_short(ctxs, K, M, N, pitch):
    """k_x3_tn's masked one-tile form (round 6: dW = Y^T (dZ ⊙ [Z > 0]) s for
    C3 / C4's aggregate-first bottom layer, M <= 128 feature rows, dense Y
    rows whose pitch covers 32 ceil(M / 32) floats — the last case's 104 does
    not and stays on the fp32-input kernel; NaN pad columns only reach output
    rows >= M, never stored): within the split path's bound of an fp64
    product, three runs each (its counted step wait once left a stale step
    about one run in four; the drained wait must not)."""
    f32, s3 = ctxs
    g = torch.Generator(device=DEV).manual_seed(K + M)
    Y = torch.full((K, pitch), float("nan"), device=DEV)[:, :M]
    Y.copy_(torch.randn(K, M, device=DEV, generator=g))
    G = torch.randn(K, N, device=DEV, generator=g)
    Z = torch.relu(torch.randn(K, N, device=DEV, generator=g))
    s = 2.0
    C32 = torch.empty(M, N, device=DEV)
    f32.gemm_tn_masked(Y, G, Z, C32, scale=s)
    Gm = torch.where(Z > 0, G.double() * s, torch.zeros_like(G, dtype=torch.float64))
    ref = Y.double().T @ Gm
    scale = Y.double().abs().T @ Gm.abs() + 1e-30
    torch.cuda.synchronize()
    e32 = ((C32.double() - ref).abs() / scale).max().item()
    for _ in range(3):
        C3 = torch.full((M, N), float("nan"), device=DEV)
        s3.gemm_tn_masked(Y, G, Z, C3, scale=s)
        torch.cuda.synchronize()
        assert not torch.isnan(C3).any()
        e3 = ((C3.double() - ref).abs() / scale).max().item()
        assert e3 <= 1.25 * e32 + 1e-7, (e3, e32)
