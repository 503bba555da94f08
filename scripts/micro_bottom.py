"""Micro benchmark of the transform-first bottom layer's planar pair-table GEMMs
at C2 size, alone on the GPU: k_h2_nn3 (H = X[src] W) and k_h2_tn4 (dW =
X[src]^T dH, per-part column maxima given) — time per call and effective
rate on the algorithmic bytes.  Timing probes (NTS_NN3_DIAG / NTS_TN4_DIAG)
exist only in the probe build of the library:

  make -C sample-based-gnn_amd/csrc probe
  NTS_HIP_LIB=scripts/probe/lib/libnts_hip.so NTS_NN3_DIAG=1 python scripts/micro_bottom.py
  python scripts/micro_bottom.py [--iters 20]
"""
import argparse
import json
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sample-based-gnn_amd"))

import torch  # noqa: E402

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
    a = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(a.V, 640, device=dev, generator=g)[:, :a.K]
    rows = torch.randperm(a.V, device=dev, generator=g)[:a.M].to(torch.int32).sort().values
    W = torch.randn(a.K, a.N, device=dev, generator=g)
    G = torch.randn(a.M, a.N, device=dev, generator=g)
    C = torch.empty(a.M, a.N, device=dev)
    dW = torch.empty(a.K, a.N, device=dev)
    h2 = HipContext(0)
    Q, rs = h2.h2_split_rows_planar(X)
    R = h2.colmax_rows_per_part(a.N)
    nparts = (a.M + R - 1) // R
    pad = torch.zeros(nparts * R, a.N, device=dev)
    pad[:a.M] = G.abs() * rs[rows.long()][:, None]  # maxima of |rs[row] G|
    parts = pad.view(nparts, R, a.N).max(1).values.contiguous().view(torch.int32)
    Kp = Q.shape[1] // 2
    row_bytes = 4 * Kp
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith("NTS_")}}
    nn = timeit(lambda: h2.gemm_h2p_gather(Q, rs, rows, W, C), a.iters)
    tn = timeit(lambda: h2.gemm_h2p_tn_gather(Q, rs, rows, G, dW, a.K, parts=parts, rows_per_part=R), a.iters)
    nn_bytes = a.M * (row_bytes + 4 + 4) + a.M * a.N * 4
    tn_bytes = a.M * (row_bytes + 4 + 4) + a.M * a.N * 4
    out["nn_us"] = round(nn, 1)
    out["nn_TBps"] = round(nn_bytes / nn / 1e6, 2)
    out["tn_us"] = round(tn, 1)
    out["tn_TBps"] = round(tn_bytes / tn / 1e6, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
