"""GEMM scaling sweep (NN): per-k-step cost and per-round cost.  GPU box only."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import torch
from nts import hip as H

def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3

ctx = H.HipContext(0, seed=1)
for (M, N, K) in [(136000, 128, 32), (136000, 128, 128), (136000, 128, 602), (136000, 128, 1204),
                  (98304, 128, 602), (98304 * 2, 128, 602), (256 * 128, 128, 602), (512 * 128, 128, 602),
                  (768 * 128, 128, 600), (768 * 128, 128, 2400)]:
    A = torch.randn(M, K, device="cuda"); B = torch.randn(K, N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    fl = 2 * M * N * K
    us = t(lambda: ctx.gemm(A, B, C))
    print(f"M={M} N={N} K={K} blocks={-(-M//128)}: NN {us:7.1f}us {fl/us/1e6:6.1f}TF", flush=True)
