"""Micro benchmark of the fused output layer + loss (nts_hip_linear_xent_train)
at the C2 top layer's shape (10,000 rows, 128 -> 41): time per call alone.

  python scripts/micro_top.py [--n 10000 --K 128 --C 41 --iters 50]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sample-based-gnn_amd"))
sys.path.insert(0, str(ROOT / "scripts"))

import torch  # noqa: E402

from micro_agg import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--C", type=int, default=41)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from nts.hip import HipContext
    hip = HipContext(0)
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(1)
    Y = torch.randn(a.n, a.K, device=dev, generator=g)
    W = torch.randn(a.K, a.C, device=dev, generator=g) * 0.1
    lab = torch.randint(0, a.C, (a.n,), device=dev, generator=g)
    loss = torch.empty((), device=dev)
    dY = torch.empty(a.n, a.K, device=dev)
    dW = torch.empty(a.K, a.C, device=dev)
    us = timeit(lambda: hip.linear_xent_train(Y, W, lab, loss, dY, dW), a.iters)
    print(json.dumps({"n": a.n, "K": a.K, "C": a.C, "train_us": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
