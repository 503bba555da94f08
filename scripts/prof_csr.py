"""Hop-1 sampling with the CSR transpose, repeated (rocprofv3 target)."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import torch  # noqa: E402

from nts import hip as H, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
g, F, C = synthetic.shaped("reddit", device=dev)
ctx = H.HipContext(0, seed=2000)
col, rows = ctx.build_csc(g.src, g.dst, g.n_vertices)
od, idg = ctx.degrees(g.src, g.dst, g.n_vertices)
G = H.DeviceGraph(g.n_vertices, g.n_edges, col, rows, idg, od)
seeds = torch.randperm(g.n_vertices, device=dev)[:10000].to(torch.int32)
caps = H.layer_caps(10000, [25, 10], g.n_vertices, g.n_edges)
ctx.reserve(g.n_vertices, max(max(c) for c in caps))
vsz = torch.tensor([10000], dtype=torch.int32, device=dev)
l0 = H.LayerBuffers(*caps[0], seeds, vsz, dev, csr=True)
ctx.sample_layer(G, l0, 25, 0, 0, 0, 0)
l1 = H.LayerBuffers(*caps[1], l0.source, l0.sizes[2:3], dev, csr=True)
for _ in range(20):
    ctx.sample_layer(G, l1, 10, 1, 0, 0, 0)
torch.cuda.synchronize()
print("ok", l1.sizes_host())
