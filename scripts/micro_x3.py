"""Micro benchmark of the fp32-exact row-gathered bottom-layer GEMMs at C2 size
(NTS_GEMM_SPLIT3; csrc/gemmx3.hip where the shape qualifies, else gemm3.hip),
alone on the GPU: time per call and the rate on the algorithmic bytes (the
gathered fp32 rows once, the other operand and the output once).

  python scripts/micro_x3.py [--iters 20]   (NTS_HIP_LIB selects a variant build)
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
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--V", type=int, default=232965)
    ap.add_argument("--M", type=int, default=228616)
    ap.add_argument("--K", type=int, default=602)
    ap.add_argument("--N", type=int, default=128)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(a.V, 640, device=dev, generator=g)[:, :a.K]
    rows = torch.randperm(a.V, device=dev, generator=g)[:a.M].to(torch.int32).sort().values
    W = torch.randn(a.K, a.N, device=dev, generator=g)
    G = torch.randn(a.M, a.N, device=dev, generator=g)
    C = torch.empty(a.M, a.N, device=dev)
    dW = torch.empty(a.K, a.N, device=dev)
    s3 = HipContext(0)
    s3.set_gemm_mode(_abi.NTS_GEMM_SPLIT3)
    byt = a.M * 4.0 * a.K + a.M * 4.0 * a.N + 4.0 * a.K * a.N
    for name, fn in (("nn_gather", lambda: s3.gemm_gather(X, rows, W, C)),
                     ("tn_gather", lambda: s3.gemm_tn_gather(X, rows, G, dW))):
        us = timeit(fn, a.iters)
        print(json.dumps({"kernel": name, "tag": a.tag, "us": round(us, 1),
                          "TBps_algorithmic": round(byt / us / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
