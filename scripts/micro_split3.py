"""Layer GEMMs of the Reddit-shaped bottom layer, fp32 MFMA vs the split-bf16
(NTS_GEMM_SPLIT3) kernels: NN + relu/dropout over Y0 (aggregate-first),
the row-gathered NN over the frontier (transform-first), and the two weight
gradients.  GPU box only."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import torch
from nts import hip as H, _abi


def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


f32 = H.HipContext(0, seed=1)
s3 = H.HipContext(0, seed=1)
s3.set_gemm_mode(_abi.NTS_GEMM_SPLIT3)
K, N = 602, 128
V = 232965
table = torch.rand(V, 608, device="cuda")[:, :K]
Ma, Mt = 136076, 228656
Y0 = torch.rand(Ma, 608, device="cuda")[:, :K]
rows = torch.randperm(V, device="cuda")[:Mt].to(torch.int32)
W = torch.randn(K, N, device="cuda") * 0.05
Ca = torch.empty(Ma, N, device="cuda")
Ct = torch.empty(Mt, N, device="cuda")
Ga = torch.randn(Ma, N, device="cuda")
Gt = torch.randn(Mt, N, device="cuda")
Xa = torch.relu(torch.randn(Ma, N, device="cuda"))
D = torch.empty(K, N, device="cuda")
for _ in range(100): f32.gemm(Y0, W, Ca)  # clocks up
for name, ctx in (("fp32", f32), ("split3", s3)):
    nn = t(lambda: ctx.gemm_relu_dropout(Y0, W, Ca, p=0.5, seed=3, offset=1))
    nng = t(lambda: ctx.gemm_gather(table, rows, W, Ct))
    tn = t(lambda: ctx.gemm_tn_masked(Y0, Ga, Xa, D, scale=2.0))
    tng = t(lambda: ctx.gemm_tn_gather(table, rows, Gt, D))
    fa, ft = 2 * Ma * N * K, 2 * Mt * N * K
    print(f"[{name}] AF NN+epi {nn:6.1f}us ({fa/nn/1e6:5.1f} TF) TN masked {tn:6.1f}us ({fa/tn/1e6:5.1f}) | "
          f"TF gather NN {nng:6.1f}us ({ft/nng/1e6:5.1f}) gather TN {tng:6.1f}us ({ft/tng/1e6:5.1f})", flush=True)
