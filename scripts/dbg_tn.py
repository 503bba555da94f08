"""Repro of the masked one-tile k_x3_tn race: the masked weight gradient at
C3's shape against fp64, repeated (argv[1] times).  The product drains each
step's DMA wait; `make variant V=cnt VFLAGS=-DNTS_X3TN_COUNTED` and
NTS_HIP_LIB=scripts/probe/lib_cnt/libnts_hip.so bring back the counted wait
that read a stale step ~1 run in 4."""
import sys, torch
sys.path.insert(0, "sample-based-gnn_amd")
from nts import _abi
from nts.hip import HipContext
DEV = torch.device("cuda:0")
f32 = HipContext(0, seed=2000)
s3 = HipContext(0, seed=2000); s3.set_gemm_mode(_abi.NTS_GEMM_SPLIT3)
K, M, N, pitch = 140390, 100, 256, 128
g = torch.Generator(device=DEV).manual_seed(K + M)
Y = torch.full((K, pitch), float("nan"), device=DEV)[:, :M]
Y.copy_(torch.randn(K, M, device=DEV, generator=g))
G = torch.randn(K, N, device=DEV, generator=g)
Z = torch.relu(torch.randn(K, N, device=DEV, generator=g))
Gm = torch.where(Z > 0, G.double() * 2.0, torch.zeros_like(G, dtype=torch.float64))
ref = Y.double().T @ Gm
scale = Y.double().abs().T @ Gm.abs() + 1e-30
def check(tag, C):
    torch.cuda.synchronize()
    err = ((C.double() - ref).abs() / scale)
    bad = (err > 1e-6).nonzero()
    print(tag, "max err %.3g" % err.max().item(), "bad", bad.shape[0], "rows", sorted(set(bad[:, 0].tolist()))[:12],
          "cols", sorted(set(bad[:, 1].tolist()))[:20], flush=True)
for it in range(3):
    C32 = torch.empty(M, N, device=DEV)
    f32.gemm_tn_masked(Y, G, Z, C32, scale=2.0)
    check("f32 %d" % it, C32)
    C3 = torch.full((M, N), float("nan"), device=DEV)
    s3.gemm_tn_masked(Y, G, Z, C3, scale=2.0)
    check("s3 %d" % it, C3)
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    C3 = torch.full((M, N), float("nan"), device=DEV)
    s3.gemm_tn_masked(Y, G, Z, C3, scale=2.0)
    check("s3-only %d" % it, C3)
