"""Probe of k_h2_nnd's epilogue cost (products-shaped bottom layer): no
activation / relu / relu+dropout, on signed and on all-positive operands (relu
then zeroes nothing), and the same three on the fp32 path for comparison.

  python scripts/h2d_epi_probe.py [--iters 30]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sample-based-gnn_amd"))
sys.path.insert(0, str(ROOT / "scripts"))

import torch  # noqa: E402

from micro_layer import timeit  # noqa: E402
from nts.hip import HipContext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(3)
    M, K, N = 140156, 100, 256
    A = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(K, N, device=dev, generator=g) * 0.1
    X = torch.empty(M, N, device=dev)
    h2 = HipContext(0)
    out = {}
    for tag, (AA, WW) in (("signed", (A, W)), ("positive", (A.abs(), W.abs()))):
        out[tag + "_noact_us"] = timeit(lambda: h2.gemm_h2d_act(AA, WW, X), a.iters)
        out[tag + "_relu_us"] = timeit(lambda: h2.gemm_h2d_act(AA, WW, X, relu_dropout=True, p=0.0), a.iters)
        out[tag + "_act_us"] = timeit(lambda: h2.gemm_h2d_act(AA, WW, X, relu_dropout=True, p=0.5, seed=1,
                                                               offset=2), a.iters)
        out[tag + "_zero_frac"] = round((X == 0).float().mean().item(), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
