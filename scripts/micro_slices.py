"""Column-sliced bottom aggregation (aggregate-first, Reddit-shaped hop 1):
the fused feature gather + aggregation over the whole 602-wide rows vs over
column slices of the feature table launched one after another (each slice's
table part fits the Infinity Cache).  GPU box only."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import torch  # noqa: E402

from nts import hip as H, synthetic  # noqa: E402


def t(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


dev = torch.device("cuda", 0)
g, F, C = synthetic.shaped("reddit", device=dev)
ctx = H.HipContext(0, seed=2000)
col, rows = ctx.build_csc(g.src, g.dst, g.n_vertices)
od, idg = ctx.degrees(g.src, g.dst, g.n_vertices)
G = H.DeviceGraph(g.n_vertices, g.n_edges, col, rows, idg, od)
feat = torch.empty(g.n_vertices, 640, device=dev)[:, :F]
feat.copy_(synthetic.features(g.n_vertices, F, device=dev))
seeds = torch.randperm(g.n_vertices, device=dev)[:10000].to(torch.int32)
caps = H.layer_caps(10000, [25, 10], g.n_vertices, g.n_edges)
ctx.reserve(g.n_vertices, max(max(c) for c in caps))
vsz = torch.tensor([10000], dtype=torch.int32, device=dev)
l0 = H.LayerBuffers(*caps[0], seeds, vsz, dev, csr=True)
ctx.sample_layer(G, l0, 25, 0, 0, 0, 0)
l1 = H.LayerBuffers(*caps[1], l0.source, l0.sizes[2:3], dev, csr=False)
ctx.sample_layer(G, l1, 10, 1, 0, 0, 0)
v1, e1, s1, _ = l1.sizes_host()
y = torch.empty(v1, 640, device=dev)[:, :F]


def agg(width):
    def run():
        for c0 in range(0, F, width):
            w = min(width, F - c0)
            ctx.spmm_csc_fwd(l1.column_offset, l1.row_indices, l1.edge_weight_forward,
                             l1.sizes[0:1], v1, feat[:, c0:c0 + w], y[:, c0:c0 + w], row_map=l1.source)
    return run


ref = None
byts = 4.0 * F * s1 + 8.0 * e1 + 4.0 * (v1 + 1) + 4.0 * F * v1 + 4.0 * s1
for width in (F, 304, 208, 160, 128, 96, 64):
    us = t(agg(width))
    torch.cuda.synchronize()
    if ref is None:
        ref = y.clone()
    same = torch.equal(y, ref)
    print(f"slices of {width:3d}: {us:7.1f} us  ({byts / us / 1e3:5.0f} GB/s algorithmic)  "
          f"bit-identical {same}", flush=True)
