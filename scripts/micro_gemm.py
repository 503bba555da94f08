"""Micro-benchmark of the layer GEMMs (MFMA kernels vs torch/hipBLASLt) at the
Reddit-shaped bottom-layer sizes.  GPU box only."""
import sys, time, pathlib
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
for (M, N, K) in [(136000, 128, 602), (225000, 128, 602), (10000, 41, 128), (136000, 41, 128)]:
    A = torch.randn(M, K, device="cuda"); B = torch.randn(K, N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    fl = 2 * M * N * K
    us = t(lambda: ctx.gemm(A, B, C)); ut = t(lambda: torch.matmul(A, B, out=C))
    G = torch.randn(M, N, device="cuda"); D = torch.empty(K, N, device="cuda")
    us2 = t(lambda: ctx.gemm(A, G, D, trans_a=True)); ut2 = t(lambda: torch.matmul(A.t(), G, out=D))
    print(f"M={M} N={N} K={K}: NN mfma {us:7.1f}us {fl/us/1e6:6.1f}TF  torch {ut:7.1f}us {fl/ut/1e6:6.1f}TF | "
          f"TN mfma {us2:7.1f}us {fl/us2/1e6:6.1f}TF torch {ut2:7.1f}us {fl/ut2/1e6:6.1f}TF", flush=True)
    if K % 32:  # 128-byte aligned row pitch (the bottom aggregation output's layout)
        Ap = torch.randn(M, (K + 31) // 32 * 32, device="cuda")[:, :K]
        us3 = t(lambda: ctx.gemm(Ap, B, C)); us4 = t(lambda: ctx.gemm(Ap, G, D, trans_a=True))
        print(f"   padded pitch {Ap.stride(0)}: NN {us3:7.1f}us {fl/us3/1e6:6.1f}TF | TN {us4:7.1f}us {fl/us4/1e6:6.1f}TF", flush=True)
