"""Layer GEMMs at the Reddit-shaped bottom layer as the bench runs them:
NN + relu/dropout epilogue (A with the 128-byte pitch) and the masked TN
weight gradient.  GPU box only; kernel variants via env (NTS_WRES_DEPTH ...)."""
import os, sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import torch
from nts import hip as H


def t(fn, it=30):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


ctx = H.HipContext(0, seed=1)
M, K, N = 136076, 602, 128
A = torch.randn(M, 640, device="cuda")[:, :K]
B = torch.randn(K, N, device="cuda")
C = torch.empty(M, N, device="cuda")
G = torch.randn(M, N, device="cuda")
D = torch.empty(K, N, device="cuda")
fl = 2 * M * N * K
ref = A @ B
for _ in range(200): ctx.gemm(A, B, C)  # clocks up
us0a = t(lambda: ctx.gemm(A, B, C))
us = t(lambda: ctx.gemm_relu_dropout(A, B, C, p=0.5, seed=3, offset=1))
us2 = t(lambda: ctx.gemm_tn_masked(A, G, C, D, scale=2.0))
us0 = t(lambda: ctx.gemm(A, B, C))
ctx.gemm(A, B, C)
torch.cuda.synchronize()
err = ((C - ref).abs().max() / ref.abs().max()).item()
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("NTS_"))
print(f"[{tag}] NN {us0a:7.1f}/{us0:7.1f}us NN+epi {us:7.1f}us {fl/us/1e6:6.1f}TF | TN masked {us2:7.1f}us {fl/us2/1e6:6.1f}TF | relerr {err:.1e}",
      flush=True)
