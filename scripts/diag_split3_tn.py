"""TN split kernel timing probes (NTS_S3_DIAG bits, results invalid)."""
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
G = torch.randn(M, N, device="cuda")
D = torch.empty(K, N, device="cuda")
for _ in range(30): s3.gemm(Y0, G, D, trans_a=True)
print(f"diag={os.environ.get('NTS_S3_DIAG', '0')}: TN {t(lambda: s3.gemm(Y0, G, D, trans_a=True)):6.1f} us", flush=True)
