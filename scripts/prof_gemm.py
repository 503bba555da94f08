"""Run each layer-GEMM kernel a few times at the Reddit bottom-layer shape (for
rocprofv3 counter passes).  GPU box only."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import torch  # noqa: E402

from nts import hip as H  # noqa: E402

ctx = H.HipContext(0, seed=1)
M, N, K = 136000, 128, 602
A = torch.randn(M, K, device="cuda")
B = torch.randn(K, N, device="cuda")
C = torch.empty(M, N, device="cuda")
G = torch.randn(M, N, device="cuda")
D = torch.empty(K, N, device="cuda")
X = torch.relu(torch.randn(M, N, device="cuda"))
for _ in range(5):
    ctx.gemm(A, B, C)
    ctx.gemm_relu_dropout(A, B, C, p=0.5, seed=1, offset=2)
    ctx.gemm(A, G, D, trans_a=True)
    ctx.gemm_tn_masked(A, G, X, D, scale=2.0)
torch.cuda.synchronize()
print("ok")
