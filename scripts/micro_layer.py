"""Micro benchmark of one dense layer's GEMMs (forward with relu/dropout,
weight gradient with the activation backward) on the layer GEMM paths, alone
on the GPU.  Default shape: the products-shaped bottom layer (C3/C4: ~140K
aggregated rows, 100 -> 256).

  python scripts/micro_layer.py [--M 140156 --K 100 --N 256] [--iters 20]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sample-based-gnn_amd"))

import torch  # noqa: E402

from nts import _abi  # noqa: E402
from nts.hip import HipContext  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / iters * 1e3, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--M", type=int, default=140156)
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--N", type=int, default=256)
    a = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(3)
    A = torch.randn(a.M, a.K, device=dev, generator=g)
    W = torch.randn(a.K, a.N, device=dev, generator=g) * 0.1
    G = torch.randn(a.M, a.N, device=dev, generator=g)
    X = torch.empty(a.M, a.N, device=dev)
    dW = torch.empty(a.K, a.N, device=dev)
    out = {"shape": [a.M, a.K, a.N]}
    for name, mode in (("f32", _abi.NTS_GEMM_F32), ("split3", _abi.NTS_GEMM_SPLIT3),
                       ("split3all", _abi.NTS_GEMM_SPLIT3_ALL)):
        c = HipContext(0)
        c.set_gemm_mode(mode)
        out[name + "_fwd_act_us"] = timeit(lambda: c.gemm_relu_dropout(A, W, X, p=0.5, seed=1, offset=2), a.iters)
        out[name + "_tn_masked_us"] = timeit(lambda: c.gemm_tn_masked(A, G, X, dW, scale=2.0), a.iters)
    h2 = HipContext(0)
    Q, rs = h2.h2_split_rows_planar(A)
    out["h2_split_us"] = timeit(lambda: h2.h2_split_rows_planar(A), a.iters)
    out["h2p_fwd_act_us"] = timeit(lambda: h2.gemm_h2p_gather(Q, rs, None, W, X, relu_dropout=True, p=0.5,
                                                               seed=1, offset=2), a.iters)
    out["h2d_fwd_act_us"] = timeit(lambda: h2.gemm_h2d_act(A, W, X, relu_dropout=True, p=0.5, seed=1,
                                                            offset=2), a.iters)
    out["h2d_fwd_relu_us"] = timeit(lambda: h2.gemm_h2d_act(A, W, X, relu_dropout=True, p=0.0), a.iters)
    out["h2d_fwd_noact_us"] = timeit(lambda: h2.gemm_h2d_act(A, W, X), a.iters)
    Kp = (a.K + 31) // 32 * 32
    Q2 = torch.empty(a.M, 2 * Kp, dtype=torch.int16, device=dev)
    rs2 = torch.empty(a.M, device=dev)
    out["h2d_fwd_act_qout_us"] = timeit(lambda: h2.gemm_h2d_act(A, W, X, relu_dropout=True, p=0.5, seed=1,
                                                                 offset=2, Q=Q2, rs=rs2), a.iters)
    out["bytes_fwd_MB"] = round((a.M * a.K + a.M * a.N) * 4 / 1e6, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
