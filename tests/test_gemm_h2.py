"""Two-piece f16 pair-table GEMMs (NTS_GEMM_H2, csrc/gemmh2.hip) vs fp64 and vs
the fp32-input MFMA path.

Bar: on the transform-first bottom layer's shapes (row-gathered NN with and
without the relu/dropout epilogue, row-gathered TN with and without the
relu/dropout backward) the pair-table path's error against an fp64 GEMM of the
same fp32 operands, normalised by |A| |B| per element, is at most 2x the fp32
MFMA path's (plus 1e-7) and below 1e-6 — rows spanning twelve decades of
magnitude and gradients of 1e-7 included (the per-row / per-column power-of-two
scales); the dropout keep mask is the fp32 path's; results are deterministic.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def ctx():
    from nts.hip import HipContext
    return HipContext(0, seed=2000)


def _check(got32, goth2, ref, scale, factor=2.0):
    e32 = ((got32.double() - ref).abs() / scale).max().item()
    eh2 = ((goth2.double() - ref).abs() / scale).max().item()
    print(f"[h2] fp32 MFMA {e32:.3e}  h2 {eh2:.3e}")
    assert eh2 <= factor * e32 + 1e-7, (eh2, e32)
    assert eh2 < 1e-6, eh2


def _table(V, K, g, decades=0.0):
    ld = (K + 31) // 32 * 32 + 32
    X = torch.full((V, ld), float("nan"), device=DEV)[:, :K]
    X.copy_(torch.randn(V, K, device=DEV, generator=g))
    if decades:
        X.mul_(10.0 ** ((torch.rand(V, 1, device=DEV, generator=g) - 0.5) * decades))
    X[3].zero_()  # an all-zero row (scale 1)
    return X


def test_split_rows_roundtrip(ctx):
    g = torch.Generator(device=DEV).manual_seed(7)
    X = _table(5000, 602, g, decades=12)
    P, rs = ctx.h2_split_rows(X)
    torch.cuda.synchronize()
    assert P.shape == (5000, 608) and (P[:, 602:] == 0).all()
    w = P.view(torch.int16).view(5000, 608, 2)
    y = w[..., 0].view(torch.float16).float() + w[..., 1].view(torch.float16).float()
    rec = y[:, :602].double() * rs.double()[:, None]
    # rs is a power of two; the row max lands in [2^14, 2^15)
    assert torch.equal(torch.frexp(rs).mantissa[rs != 0], torch.full_like(rs[rs != 0], 0.5))
    m = y[:, :602].abs().max(1).values
    nz = m > 0
    assert ((m[nz] >= 2 ** 14) & (m[nz] < 2 ** 15)).all()
    rmax = X.double().abs().max(1).values[:, None] + 1e-300
    assert ((rec - X.double()).abs() <= 2.0 ** -23 * X.double().abs() + 2.0 ** -38 * rmax).all()


@pytest.mark.parametrize("M,N,K,decades", [(228656, 128, 602, 0), (3000, 128, 602, 12),
                                           (2500, 256, 100, 6), (300, 16, 64, 0)])
def test_h2_gemm_gather(ctx, M, N, K, decades):
    g = torch.Generator(device=DEV).manual_seed(M + K + N)
    V = M + M // 3 + 11
    X = _table(V, K, g, decades)
    rows = torch.randperm(V, device=DEV, generator=g)[:M].to(torch.int32)
    rows[5] = 3  # the zero row
    W = torch.randn(K, N, device=DEV, generator=g) * 0.05
    P, rs = ctx.h2_split_rows(X)
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.full((M, N), float("nan"), device=DEV)
    ctx.gemm_gather(X, rows, W, C32)
    ctx.gemm_h2_gather(P, rs, rows, W, Ch)
    Xg = X[rows.long()].double()
    ref = Xg @ W.double()
    scale = Xg.abs() @ W.double().abs() + 1e-300
    torch.cuda.synchronize()
    assert not torch.isnan(Ch).any()
    _check(C32, Ch, ref, scale)
    Ch2 = torch.empty_like(Ch)
    ctx.gemm_h2_gather(P, rs, rows, W, Ch2)
    torch.cuda.synchronize()
    assert torch.equal(Ch, Ch2)


def test_h2_gemm_all_rows(ctx):
    g = torch.Generator(device=DEV).manual_seed(11)
    X = _table(4099, 301, g)
    W = torch.randn(301, 128, device=DEV, generator=g)
    P, rs = ctx.h2_split_rows(X)
    C32 = torch.empty(4099, 128, device=DEV)
    Ch = torch.empty(4099, 128, device=DEV)
    ctx.gemm(X, W, C32)
    ctx.gemm_h2_gather(P, rs, None, W, Ch)
    ref = X.double() @ W.double()
    scale = X.double().abs() @ W.double().abs() + 1e-300
    torch.cuda.synchronize()
    _check(C32, Ch, ref, scale)


@pytest.mark.parametrize("M,N,K,p", [(136076, 128, 602, 0.5), (2050, 64, 77, 0.2), (1000, 128, 128, 0.0)])
def test_h2_relu_dropout_epilogue(ctx, M, N, K, p):
    g = torch.Generator(device=DEV).manual_seed(M + N + K + 1)
    X = _table(M, K, g)
    W = torch.randn(K, N, device=DEV, generator=g)
    P, rs = ctx.h2_split_rows(X)
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.empty(M, N, device=DEV)
    seed, offset = 0x1234_5678_9ABC, 77
    ctx.gemm_relu_dropout(X, W, C32, p=p, seed=seed, offset=offset)
    ctx.gemm_h2_gather(P, rs, None, W, Ch, relu_dropout=True, p=p, seed=seed, offset=offset)
    Z = X.double() @ W.double()
    scale = X.double().abs() @ W.double().abs() + 1e-300
    torch.cuda.synchronize()
    clear = Z.abs() > 1e-5 * scale
    assert torch.equal((C32 != 0) & clear, (Ch != 0) & clear)
    s = 1.0 / (1.0 - p)
    ref = torch.where(C32 != 0, torch.relu(Z) * s, torch.zeros_like(Z))
    e32 = ((C32.double() - ref).abs() / (scale * s))[clear].max().item()
    eh = ((Ch.double() - ref).abs() / (scale * s))[clear].max().item()
    assert eh <= 2.0 * e32 + 1e-7 and eh < 1e-6, (eh, e32)


@pytest.mark.parametrize("M,N,K,gscale", [(602, 128, 228656, 1e-7), (602, 128, 5000, 1.0),
                                          (100, 256, 3000, 1e3), (41, 64, 300, 1.0)])
def test_h2_gemm_tn_gather(ctx, M, N, K, gscale):
    g = torch.Generator(device=DEV).manual_seed(M * N + K + 9)
    V = K + K // 2 + 5
    X = _table(V, M, g, decades=6)
    rows = torch.randint(0, V, (K,), device=DEV, generator=g).to(torch.int32)
    G = torch.randn(K, N, device=DEV, generator=g) * gscale
    G[:, 5] *= 1e-9  # a column far below the others
    P, rs = ctx.h2_split_rows(X)
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.full((M, N), float("nan"), device=DEV)
    ctx.gemm_tn_gather(X, rows, G, C32)
    ctx.gemm_h2_tn_gather(P, rs, rows, G, Ch, M)
    Xg = X[rows.long()].double()
    ref = Xg.t() @ G.double()
    scale = Xg.abs().t() @ G.double().abs() + 1e-300
    torch.cuda.synchronize()
    assert not torch.isnan(Ch).any()
    _check(C32, Ch, ref, scale)
    Ch2 = torch.empty_like(Ch)
    ctx.gemm_h2_tn_gather(P, rs, rows, G, Ch2, M)
    torch.cuda.synchronize()
    assert torch.equal(Ch, Ch2)


@pytest.mark.parametrize("M,N,K", [(602, 128, 135758), (602, 128, 5000)])
def test_h2_gemm_tn_masked(ctx, M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M * 3 + N + K)
    A = _table(K, M, g)
    G = torch.randn(K, N, device=DEV, generator=g) * 1e-5
    Xm = torch.relu(torch.randn(K, N, device=DEV, generator=g))
    P, rs = ctx.h2_split_rows(A)
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.empty(M, N, device=DEV)
    ctx.gemm_tn_masked(A, G, Xm, C32, scale=2.0)
    ctx.gemm_h2_tn_gather(P, rs, None, G, Ch, M, X=Xm, bscale=2.0)
    Bm = G.double() * (Xm > 0).double() * 2.0
    ref = A.double().t() @ Bm
    scale = A.double().abs().t() @ Bm.abs() + 1e-300
    torch.cuda.synchronize()
    _check(C32, Ch, ref, scale)


def test_h2_error_distribution_report(ctx):
    """C2 transform-first shape: mean and max normalised error of both paths."""
    g = torch.Generator(device=DEV).manual_seed(42)
    X = torch.rand(228656, 608, device=DEV, generator=g)[:, :602]
    W = torch.randn(602, 128, device=DEV, generator=g) * 0.05
    P, rs = ctx.h2_split_rows(X)
    C32 = torch.empty(228656, 128, device=DEV)
    Ch = torch.empty_like(C32)
    ctx.gemm(X, W, C32)
    ctx.gemm_h2_gather(P, rs, None, W, Ch)
    ref = X.double() @ W.double()
    scale = X.double().abs() @ W.double().abs() + 1e-300
    torch.cuda.synchronize()
    r32 = (C32.double() - ref).abs() / scale
    rh = (Ch.double() - ref).abs() / scale
    print(f"\n[h2] fp32 MFMA: mean {r32.mean().item():.3e} max {r32.max().item():.3e}; "
          f"h2: mean {rh.mean().item():.3e} max {rh.max().item():.3e}")


def test_split_rows_planar_matches_pairs(ctx):
    g = torch.Generator(device=DEV).manual_seed(8)
    X = _table(3000, 602, g, decades=8)
    P, rs = ctx.h2_split_rows(X)
    Q, rs2 = ctx.h2_split_rows_planar(X)
    torch.cuda.synchronize()
    assert torch.equal(rs, rs2)
    w = P.view(torch.int16).view(3000, 608, 2)
    assert torch.equal(Q[:, :608], w[..., 0]) and torch.equal(Q[:, 608:], w[..., 1])


@pytest.mark.parametrize("M,N,K,gscale", [(602, 128, 228656, 1e-7), (602, 128, 5003, 1.0),
                                          (100, 256, 3000, 1e3), (600, 128, 100, 1.0),
                                          (41, 128, 17, 1.0)])
def test_h2p_gemm_tn_gather(ctx, M, N, K, gscale):
    """TN v3 on the planar table: whole rows by LDS DMA, every output row in one block."""
    g = torch.Generator(device=DEV).manual_seed(M * N + K + 19)
    V = K + K // 2 + 5
    X = _table(V, M, g, decades=6)
    rows = torch.randint(0, V, (K,), device=DEV, generator=g).to(torch.int32)
    G = torch.randn(K, N, device=DEV, generator=g) * gscale
    G[:, 5] *= 1e-9
    Q, rs = ctx.h2_split_rows_planar(X)
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.full((M, N), float("nan"), device=DEV)
    ctx.gemm_tn_gather(X, rows, G, C32)
    ctx.gemm_h2p_tn_gather(Q, rs, rows, G, Ch, M)
    Xg = X[rows.long()].double()
    ref = Xg.t() @ G.double()
    scale = Xg.abs().t() @ G.double().abs() + 1e-300
    torch.cuda.synchronize()
    assert not torch.isnan(Ch).any()
    _check(C32, Ch, ref, scale)
    Ch2 = torch.empty_like(Ch)
    ctx.gemm_h2p_tn_gather(Q, rs, rows, G, Ch2, M)
    torch.cuda.synchronize()
    assert torch.equal(Ch, Ch2)


@pytest.mark.parametrize("M,N,K,gscale,anti", [(602, 128, 228656, 1e-7, False),
                                               (602, 128, 5003, 1.0, False),
                                               (100, 256, 3000, 1e3, False), (41, 128, 17, 1.0, False),
                                               (602, 128, 5003, 1.0, True),
                                               (602, 128, 228656, 1e-3, True)])
def test_h2p_gemm_tn_gather_given_column_maxima(ctx, M, N, K, gscale, anti):
    """TN v4 with the per-part column maxima of |rs[row] B| given (the CSR
    backward's epilogue) instead of its per-chunk pre-pass over B: the same
    error bar vs fp64, deterministic.  anti: B's rows scaled inversely to the
    magnitudes of their X rows (6 decades), where max |rs| x max |B| would
    overstate the operand maxima by ~2^20."""
    g = torch.Generator(device=DEV).manual_seed(M * N + K + 23)
    V = K + K // 2 + 5
    X = _table(V, M, g, decades=6)
    rows = torch.randint(0, V, (K,), device=DEV, generator=g).to(torch.int32)
    G = torch.randn(K, N, device=DEV, generator=g) * gscale
    if anti:
        amax = X[rows.long()].abs().amax(1, keepdim=True)
        G *= torch.where(amax > 0, 1.0 / amax.clamp_min(1e-30), torch.ones_like(amax))
    G[:, 5] *= 1e-9
    G[:, 9] = 0.0  # an all-zero column (max 0)
    Q, rs = ctx.h2_split_rows_planar(X)
    R = 8  # rows per part (the CSR backward's for N = 128)
    nparts = (K + R - 1) // R
    pad = torch.zeros(nparts * R, N, device=DEV)
    pad[:K] = G.abs() * rs[rows.long()][:, None]  # maxima of |rs[row] G[k, c]|
    cm = pad.view(nparts, R, N).max(1).values.contiguous().view(torch.int32)
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.full((M, N), float("nan"), device=DEV)
    ctx.gemm_tn_gather(X, rows, G, C32)
    ctx.gemm_h2p_tn_gather(Q, rs, rows, G, Ch, M, parts=cm, rows_per_part=R)
    Xg = X[rows.long()].double()
    ref = Xg.t() @ G.double()
    scale = Xg.abs().t() @ G.double().abs() + 1e-300
    torch.cuda.synchronize()
    assert not torch.isnan(Ch).any()
    assert (Ch[:, 9] == 0).all()
    _check(C32, Ch, ref, scale)
    Ch2 = torch.empty_like(Ch)
    ctx.gemm_h2p_tn_gather(Q, rs, rows, G, Ch2, M, parts=cm, rows_per_part=R)
    torch.cuda.synchronize()
    assert torch.equal(Ch, Ch2)


@pytest.mark.parametrize("M,N,K,decades,tail", [(228656, 128, 602, 0, False), (3001, 128, 602, 12, False),
                                                (2500, 256, 100, 6, False), (17, 128, 64, 0, False),
                                                (228656, 128, 602, 0, True), (3001, 128, 602, 12, True),
                                                (17, 128, 602, 3, True), (5000, 256, 600, 6, True)])
def test_h2p_gemm_gather(ctx, M, N, K, decades, tail):
    """NN v3 on the planar table (W slices in registers, whole rows by LDS DMA);
    tail: rows padded to 2560 bytes with the row scale in the tail — the
    four-stage NN v4 (Kp 608: 19 steps), bit-identical to v3."""
    g = torch.Generator(device=DEV).manual_seed(M + K + N + 3)
    V = M + M // 3 + 11
    X = _table(V, K, g, decades)
    rows = torch.randperm(V, device=DEV, generator=g)[:M].to(torch.int32)
    rows[min(5, M - 1)] = 3
    W = torch.randn(K, N, device=DEV, generator=g) * 0.05
    Q, rs = ctx.h2_split_rows_planar(X, tail=tail)
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.full((M, N), float("nan"), device=DEV)
    ctx.gemm_gather(X, rows, W, C32)
    ctx.gemm_h2p_gather(Q, rs, rows, W, Ch)
    if tail:  # v4 (row scales from the tails) == v3 (row scales from rs), bit for bit
        Q3, rs3 = ctx.h2_split_rows_planar(X)
        assert torch.equal(Q3, Q) and torch.equal(rs3, rs)
        C3 = torch.full((M, N), float("nan"), device=DEV)
        ctx.gemm_h2p_gather(Q3, rs3, rows, W, C3)
        torch.cuda.synchronize()
        assert torch.equal(C3, Ch)
    Xg = X[rows.long()].double()
    ref = Xg @ W.double()
    scale = Xg.abs() @ W.double().abs() + 1e-300
    torch.cuda.synchronize()
    assert not torch.isnan(Ch).any()
    _check(C32, Ch, ref, scale)
    P, rs1 = ctx.h2_split_rows(X)
    Ci = torch.empty_like(Ch)
    ctx.gemm_h2_gather(P, rs1, rows, W, Ci)  # the interleaved kernel: same products, same sums
    torch.cuda.synchronize()
    assert torch.equal(Ch, Ci)


@pytest.mark.parametrize("p", [0.5, 0.0])
def test_h2p_relu_dropout_epilogue(ctx, p):
    M, N, K = 20000, 128, 602
    g = torch.Generator(device=DEV).manual_seed(99)
    X = _table(M, K, g)
    W = torch.randn(K, N, device=DEV, generator=g)
    Q, rs = ctx.h2_split_rows_planar(X)
    P, rs1 = ctx.h2_split_rows(X)
    Ch = torch.empty(M, N, device=DEV)
    Ci = torch.empty(M, N, device=DEV)
    seed, offset = 0x1234_5678_9ABC, 77
    ctx.gemm_h2p_gather(Q, rs, None, W, Ch, relu_dropout=True, p=p, seed=seed, offset=offset)
    ctx.gemm_h2_gather(P, rs1, None, W, Ci, relu_dropout=True, p=p, seed=seed, offset=offset)
    torch.cuda.synchronize()
    assert torch.equal(Ch, Ci)


@pytest.mark.parametrize("M,N,K,decades", [(140156, 256, 100, 0), (5003, 128, 128, 12),
                                           (4099, 256, 96, 6), (777, 256, 4, 0), (33, 128, 64, 3)])
def test_h2d_gemm_dynamic_input(ctx, M, N, K, decades):
    """The narrow dynamic-input NN (k_h2_nnd: A split into pairs in the
    kernel): the pair-table error bar vs fp64, deterministic, and the pair
    table it writes on the way equal to h2_split_rows_planar's bit for bit."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K + 41)
    X = _table(M, K, g, decades)
    W = torch.randn(K, N, device=DEV, generator=g) * 0.05
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.full((M, N), float("nan"), device=DEV)
    ctx.gemm(X, W, C32)
    Kp = (K + 31) // 32 * 32
    Q = torch.full((M, 2 * Kp), -1, dtype=torch.int16, device=DEV)
    rs = torch.full((M,), float("nan"), device=DEV)
    ctx.gemm_h2d_act(X, W, Ch, Q=Q, rs=rs)
    ref = X.double() @ W.double()
    scale = X.double().abs() @ W.double().abs() + 1e-300
    Q0, rs0 = ctx.h2_split_rows_planar(X)
    Ch2 = torch.empty_like(Ch)
    ctx.gemm_h2d_act(X, W, Ch2)
    torch.cuda.synchronize()
    assert not torch.isnan(Ch).any()
    _check(C32, Ch, ref, scale)
    assert torch.equal(Ch, Ch2)
    assert torch.equal(Q, Q0[:, :2 * Kp]) and torch.equal(rs, rs0)


@pytest.mark.parametrize("M,N,K,p", [(140156, 256, 100, 0.5), (2050, 128, 64, 0.2), (1000, 256, 128, 0.0)])
def test_h2d_relu_dropout_epilogue(ctx, M, N, K, p):
    """k_h2_nnd's relu/dropout epilogue drops the elements the fp32 path drops."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K + 43)
    X = _table(M, K, g)
    W = torch.randn(K, N, device=DEV, generator=g)
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.empty(M, N, device=DEV)
    seed, offset = 0x1234_5678_9ABC, 77
    ctx.gemm_relu_dropout(X, W, C32, p=p, seed=seed, offset=offset)
    ctx.gemm_h2d_act(X, W, Ch, relu_dropout=True, p=p, seed=seed, offset=offset)
    Z = X.double() @ W.double()
    scale = X.double().abs() @ W.double().abs() + 1e-300
    torch.cuda.synchronize()
    clear = Z.abs() > 1e-5 * scale
    assert torch.equal((C32 != 0) & clear, (Ch != 0) & clear)
    s = 1.0 / (1.0 - p)
    ref = torch.where(C32 != 0, torch.relu(Z) * s, torch.zeros_like(Z))
    e32 = ((C32.double() - ref).abs() / (scale * s))[clear].max().item()
    eh = ((Ch.double() - ref).abs() / (scale * s))[clear].max().item()
    assert eh <= 2.0 * e32 + 1e-7 and eh < 1e-6, (eh, e32)


def _inrow_table(V, K, g, decades):
    """Rows whose ELEMENTS span `decades` decades of magnitude (log-uniform per
    element), signs random: the dynamic range sits inside each row, where the
    per-row power-of-two scale cannot help the small elements."""
    ld = (K + 31) // 32 * 32 + 32
    X = torch.full((V, ld), float("nan"), device=DEV)[:, :K]
    mag = 10.0 ** ((torch.rand(V, K, device=DEV, generator=g) - 0.5) * decades)
    sgn = torch.where(torch.rand(V, K, device=DEV, generator=g) < 0.5, -1.0, 1.0)
    X.copy_(mag * sgn)
    return X


@pytest.mark.parametrize("decades", [10, 14])
def test_h2p_within_row_dynamic_range(ctx, decades):
    """Verdict r03 weak #2: elements spanning >= 10 decades WITHIN each row.
    (1) normwise (error / (|X| |W|), the metric of every test above): the pair
    tables stay within 2x of the fp32 MFMA path, NN (k_h2_nn3) and TN (k_h2_tn4).
    (2) the representation bound: every element carries 22 significant bits or
    an absolute error <= 2^-39 of its row's largest |x| (csrc/gemmh2.hip header),
    so |C - ref| <= 2^-21 |X||W| + 2^-38 rowmax(|X|) (1 |W|) + the fp32
    accumulation.  (3) measured and printed, not a bar: outputs that only the
    small elements feed (W zero on the columns that hold each row's large
    elements) — there the pair table's error relative to those small terms is
    far above fp32's (the fp32-exact transform-first secondary of
    bench.py is the reference-width measurement)."""
    M, N, K = 20000, 128, 602
    g = torch.Generator(device=DEV).manual_seed(decades + 101)
    V = M + 77
    X = _inrow_table(V, K, g, decades)
    rows = torch.randperm(V, device=DEV, generator=g)[:M].to(torch.int32)
    W = torch.randn(K, N, device=DEV, generator=g) * 0.05
    Q, rs = ctx.h2_split_rows_planar(X)
    Xg = X[rows.long()].double()
    scale = Xg.abs() @ W.double().abs() + 1e-300
    # (1) + (2), NN
    C32 = torch.empty(M, N, device=DEV)
    Ch = torch.full((M, N), float("nan"), device=DEV)
    ctx.gemm_gather(X, rows, W, C32)
    ctx.gemm_h2p_gather(Q, rs, rows, W, Ch)
    ref = Xg @ W.double()
    torch.cuda.synchronize()
    _check(C32, Ch, ref, scale)
    rowmax = Xg.abs().amax(1, keepdim=True)
    bound = 2.0 ** -21 * scale + 2.0 ** -38 * rowmax * W.double().abs().sum(0, keepdim=True) \
        + K * 2.0 ** -24 * scale
    assert ((Ch.double() - ref).abs() <= bound).all()
    # (1), TN: dW = X[rows]^T G with well-scaled G
    G = torch.randn(M, N, device=DEV, generator=g)
    D32 = torch.empty(K, N, device=DEV)
    Dh = torch.full((K, N), float("nan"), device=DEV)
    ctx.gemm_tn_gather(X, rows, G, D32)
    ctx.gemm_h2p_tn_gather(Q, rs, rows, G, Dh, K)
    reft = Xg.t() @ G.double()
    scalet = Xg.abs().t() @ G.double().abs() + 1e-300
    torch.cuda.synchronize()
    _check(D32, Dh, reft, scalet)
    # (3) small-only outputs: per row the columns above its median magnitude
    # get weight 0 through a row-dependent mask folded into X (W kept dense)
    med = Xg.abs().median(1, keepdim=True).values
    Xs = torch.where(Xg.abs() <= med, Xg, torch.zeros_like(Xg))
    Xbig = X.clone()
    Xbig[rows.long()] = Xs.float()
    ref_s = Xs @ W.double()
    scale_s = Xs.abs() @ W.double().abs() + 1e-300
    # the same small elements, but the pair table still scaled by the full rows
    Qs = Q.clone()
    keep = torch.zeros(V, K, dtype=torch.bool, device=DEV)
    keep[rows.long()] = Xg.abs() <= med
    Kp = Q.shape[1] // 2
    kp = torch.zeros(V, Kp, dtype=torch.bool, device=DEV)
    kp[:, :K] = keep
    Qs[:, :Kp] = torch.where(kp, Q[:, :Kp], torch.zeros_like(Q[:, :Kp]))
    Qs[:, Kp:] = torch.where(kp, Q[:, Kp:], torch.zeros_like(Q[:, Kp:]))
    Cs = torch.empty(M, N, device=DEV)
    ctx.gemm_h2p_gather(Qs, rs, rows, W, Cs)
    Cs32 = torch.empty(M, N, device=DEV)
    ctx.gemm_gather(Xbig, rows, W, Cs32)
    torch.cuda.synchronize()
    es = ((Cs.double() - ref_s).abs() / scale_s).max().item()
    es32 = ((Cs32.double() - ref_s).abs() / scale_s).max().item()
    print(f"[h2 in-row {decades} decades] small-only outputs: pair table {es:.3e}, fp32 MFMA {es32:.3e}")
    assert es32 < 1e-6
