"""Short driver for rocprofv3 passes over the split-bf16 GEMMs (C2 shapes):
5 launches each of NN+epilogue, gathered NN, TN masked, gathered TN."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import torch
from nts import hip as H, _abi

mode = _abi.NTS_GEMM_SPLIT3 if (len(sys.argv) < 2 or sys.argv[1] != "f32") else _abi.NTS_GEMM_F32
ctx = H.HipContext(0, seed=1)
ctx.set_gemm_mode(mode)
K, N, V, Ma, Mt = 602, 128, 232965, 136076, 228656
table = torch.rand(V, 608, device="cuda")[:, :K]
Y0 = torch.rand(Ma, 608, device="cuda")[:, :K]
rows = torch.randperm(V, device="cuda")[:Mt].to(torch.int32)
W = torch.randn(K, N, device="cuda") * 0.05
Ca, Ct = torch.empty(Ma, N, device="cuda"), torch.empty(Mt, N, device="cuda")
Ga, Gt = torch.randn(Ma, N, device="cuda"), torch.randn(Mt, N, device="cuda")
Xa = torch.relu(torch.randn(Ma, N, device="cuda"))
D = torch.empty(K, N, device="cuda")
for _ in range(5):
    ctx.gemm_relu_dropout(Y0, W, Ca, p=0.5, seed=3, offset=1)
    ctx.gemm_gather(table, rows, W, Ct)
    ctx.gemm_tn_masked(Y0, Ga, Xa, D, scale=2.0)
    ctx.gemm_tn_gather(table, rows, Gt, D)
torch.cuda.synchronize()
print("ok")
