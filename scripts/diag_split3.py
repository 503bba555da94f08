"""NN split kernel timing probes (NTS_S3_DIAG bits, results invalid): run one
configuration per process, print its time."""
import os, sys, pathlib
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


s3 = H.HipContext(0, seed=1)
s3.set_gemm_mode(_abi.NTS_GEMM_SPLIT3)
K, N, M = 602, 128, 136076
Y0 = torch.rand(M, 608, device="cuda")[:, :K]
W = torch.randn(K, N, device="cuda") * 0.05
C = torch.empty(M, N, device="cuda")
for _ in range(30): s3.gemm(Y0, W, C)
print(f"diag={os.environ.get('NTS_S3_DIAG', '0')}: NN {t(lambda: s3.gemm(Y0, W, C)):6.1f} us", flush=True)
