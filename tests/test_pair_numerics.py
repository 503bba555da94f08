"""CPU check of the f16 pair-table arithmetic (csrc/gemmh2.hip),
restated in numpy: the split y0 = f16(y), y1 = f16(y - y0) of a row scaled
into [2^14, 2^15), its reconstruction bound, and the three-product dot
product against fp64 — the error analysis the GPU kernels rely on
(tests/test_gemm_h2.py measures the kernels themselves on the MI355X)."""
import numpy as np


def _split(x):
    """per row: scale exponent e (max |x| 2^e in [2^14, 2^15)), pieces y0, y1"""
    m = np.abs(x).max(axis=1, keepdims=True)
    _, ex = np.frexp(m)
    e = np.where(m > 0, 15 - ex, 0)
    y = np.ldexp(x.astype(np.float32), e).astype(np.float32)
    y0 = y.astype(np.float16)
    y1 = (y - y0.astype(np.float32)).astype(np.float16)
    return e, y, y0, y1


def test_row_scale_and_reconstruction():
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((2000, 602)) *
         10.0 ** rng.uniform(-6, 6, size=(2000, 1))).astype(np.float32)
    x[7] = 0.0
    e, y, y0, y1 = _split(x)
    m = np.abs(y).max(axis=1)
    nz = m > 0
    assert ((m[nz] >= 2.0 ** 14) & (m[nz] < 2.0 ** 15)).all()
    # y - y0 is exact in fp32
    r = y.astype(np.float64) - y0.astype(np.float64)
    assert np.array_equal(r, (y - y0.astype(np.float32)).astype(np.float64))
    rec = y0.astype(np.float64) + y1.astype(np.float64)
    err = np.abs(rec - y.astype(np.float64))
    # 22 significant bits for normal y1, 2^-25 absolute (y units) below
    assert (err <= np.maximum(2.0 ** -23 * np.abs(y), 2.0 ** -25)).all()


def test_three_products_vs_fp64():
    """sum_k a0 b0 + a0 b1 + a1 b0 (each product exact, fp32 accumulation)
    against fp64, normalised by sum |a||b|: at the level of an fp32 dot
    product of the same length."""
    rng = np.random.default_rng(5)
    K, M, N = 608, 64, 32
    A = rng.standard_normal((M, K)).astype(np.float32)
    B = (rng.standard_normal((K, N)) * 0.05).astype(np.float32)
    ea, _, a0, a1 = _split(A)
    eb, _, b0, b1 = _split(B.T)  # column scales of B
    a0, a1 = a0.astype(np.float32), a1.astype(np.float32)
    b0, b1 = b0.astype(np.float32).T, b1.astype(np.float32).T
    acc = np.zeros((M, N), np.float32)
    for k in range(K):  # fp32 accumulation in k order, products exact in fp32
        acc += np.outer(a1[:, k], b0[k]) + np.outer(a0[:, k], b1[k])
        acc += np.outer(a0[:, k], b0[k])
    C = np.ldexp(np.ldexp(acc, -ea), -eb.T)
    ref = A.astype(np.float64) @ B.astype(np.float64)
    scale = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64)
    f32 = np.zeros((M, N), np.float32)
    for k in range(K):
        f32 += np.outer(A[:, k], B[k])
    e_pair = (np.abs(C - ref) / scale).max()
    e_f32 = (np.abs(f32 - ref) / scale).max()
    assert e_pair <= 2.0 * e_f32 + 1e-7, (e_pair, e_f32)
    assert e_pair < 1e-6
