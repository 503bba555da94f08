"""Where do the split GEMMs spend their time?  Same shapes with the A rows
gathered from a 64-row (L2-resident) block vs random rows of the table."""
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
K, N, V, M = 602, 128, 232965, 136076
table = torch.rand(V, 608, device="cuda")[:, :K]
rnd = torch.randperm(V, device="cuda")[:M].to(torch.int32)
seq = torch.arange(M, device="cuda", dtype=torch.int32)
hot = (torch.arange(M, device="cuda", dtype=torch.int32) % 64)
W = torch.randn(K, N, device="cuda") * 0.05
C = torch.empty(M, N, device="cuda")
G = torch.randn(M, N, device="cuda")
D = torch.empty(K, N, device="cuda")
for _ in range(50): f32.gemm_gather(table, rnd, W, C)
for name, ctx in (("fp32", f32), ("split3", s3)):
    r = {k: t(lambda: ctx.gemm_gather(table, rows, W, C)) for k, rows in (("rnd", rnd), ("seq", seq), ("hot", hot))}
    q = {k: t(lambda: ctx.gemm_tn_gather(table, rows, G, D)) for k, rows in (("rnd", rnd), ("seq", seq), ("hot", hot))}
    print(f"[{name}] NN gather rnd {r['rnd']:6.1f} seq {r['seq']:6.1f} hot {r['hot']:6.1f} | "
          f"TN gather rnd {q['rnd']:6.1f} seq {q['seq']:6.1f} hot {q['hot']:6.1f} us", flush=True)
