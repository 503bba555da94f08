"""Run a few NN GEMMs at one shape (for PMC collection).  GPU box only."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import torch
from nts import hip as H
M, N, K = (int(x) for x in sys.argv[1:4])
ta = len(sys.argv) > 4 and sys.argv[4] == "tn"
ctx = H.HipContext(0, seed=1)
A = torch.randn(M, K, device="cuda"); B = torch.randn((M if ta else K), N, device="cuda")
C = torch.empty((K if ta else M), N, device="cuda")
for _ in range(5):
    ctx.gemm(A, B, C, trans_a=ta)
torch.cuda.synchronize()
