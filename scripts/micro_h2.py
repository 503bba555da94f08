"""Micro benchmark: the transform-first bottom layer's gathered GEMMs at C2
size on the three GEMM paths (fp32 MFMA, split-bf16, f16 pair table).

  python scripts/micro_h2.py [--iters 20]
"""
import argparse
import sys
import pathlib

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
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--V", type=int, default=232965)
    ap.add_argument("--M", type=int, default=228656)
    ap.add_argument("--K", type=int, default=602)
    ap.add_argument("--N", type=int, default=128)
    a = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(a.V, 640, device=dev, generator=g)[:, :a.K]
    rows = torch.randperm(a.V, device=dev, generator=g)[:a.M].to(torch.int32)
    rows = rows.sort().values
    W = torch.randn(a.K, a.N, device=dev, generator=g)
    G = torch.randn(a.M, a.N, device=dev, generator=g)
    C = torch.empty(a.M, a.N, device=dev)
    dW = torch.empty(a.K, a.N, device=dev)
    f32 = HipContext(0)
    s3 = HipContext(0)
    s3.set_gemm_mode(_abi.NTS_GEMM_SPLIT3)
    h2 = HipContext(0)
    P, rs = h2.h2_split_rows(X)
    fl = 2.0 * a.M * a.K * a.N
    res = {}
    for name, c in (("f32", f32), ("split3", s3)):
        res[name + "_nn"] = timeit(lambda: c.gemm_gather(X, rows, W, C), a.iters)
        res[name + "_tn"] = timeit(lambda: c.gemm_tn_gather(X, rows, G, dW), a.iters)
    res["h2_nn"] = timeit(lambda: h2.gemm_h2_gather(P, rs, rows, W, C), a.iters)
    res["h2_tn"] = timeit(lambda: h2.gemm_h2_tn_gather(P, rs, rows, G, dW, a.K), a.iters)
    Q, rs2 = h2.h2_split_rows_planar(X)
    res["h2p_nn"] = timeit(lambda: h2.gemm_h2p_gather(Q, rs2, rows, W, C), a.iters)
    res["h2p_tn"] = timeit(lambda: h2.gemm_h2p_tn_gather(Q, rs2, rows, G, dW, a.K), a.iters)
    res["h2_split_rows"] = timeit(lambda: h2.h2_split_rows(X), 3)
    for k, us in res.items():
        extra = "" if "split_rows" in k else f"  {fl / us / 1e6:.1f} TF/s"
        print(f"{k:14s} {us:8.1f} us{extra}", flush=True)


if __name__ == "__main__":
    main()
