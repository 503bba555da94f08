"""Micro-benchmark of the hop-1 (bottom) layer pieces on a Reddit-shaped batch:
reference order (602-d gather+aggregate, then GEMMs) vs transform-first
(gathered GEMM, then 128-d aggregation).  GPU box only."""
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import numpy as np  # noqa: E402
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
feat = synthetic.features(g.n_vertices, F, device=dev)
seeds = torch.randperm(g.n_vertices, device=dev)[:10000].to(torch.int32)
caps = H.layer_caps(10000, [25, 10], g.n_vertices, g.n_edges)
ctx.reserve(g.n_vertices, max(max(c) for c in caps))
vsz = torch.tensor([10000], dtype=torch.int32, device=dev)
l0 = H.LayerBuffers(*caps[0], seeds, vsz, dev, csr=True)
ctx.sample_layer(G, l0, 25, 0, 0, 0, 0)
l1c = H.LayerBuffers(*caps[1], l0.source, l0.sizes[2:3], dev, csr=True)
l1n = H.LayerBuffers(*caps[1], l0.source, l0.sizes[2:3], dev, csr=False)
us_s_csr = t(lambda: ctx.sample_layer(G, l1c, 10, 1, 0, 0, 0))
us_s = t(lambda: ctx.sample_layer(G, l1n, 10, 1, 0, 0, 0))
v1, e1, s1, _ = l1c.sizes_host()
print(f"hop-1: v={v1} e={e1} s={s1}; sample {us_s:.1f} us, with CSR {us_s_csr:.1f} us")
l1 = l1c
y602 = torch.empty(v1, F, device=dev)
us_g = t(lambda: ctx.spmm_csc_fwd(l1.column_offset, l1.row_indices, l1.edge_weight_forward,
                                  l1.sizes[0:1], v1, feat, y602, row_map=l1.source))
byts = 4.0 * F * s1 + 8.0 * e1 + 4.0 * (v1 + 1) + 4.0 * F * v1 + 4.0 * s1
print(f"gather+agg 602: {us_g:.1f} us  ({byts / us_g / 1e3:.0f} GB/s algorithmic)")
featp = torch.empty(g.n_vertices, 608, device=dev)[:, :F]
featp.copy_(feat)
y602p = torch.empty(v1, 608, device=dev)[:, :F]
us_gp = t(lambda: ctx.spmm_csc_fwd(l1.column_offset, l1.row_indices, l1.edge_weight_forward,
                                   l1.sizes[0:1], v1, featp, y602p, row_map=l1.source))
print(f"gather+agg 602 from a 128-B aligned table (pitch 608), padded output: {us_gp:.1f} us")
featp4 = torch.empty(g.n_vertices, 608, device=dev)
featp4[:, :F].copy_(feat)
featp4[:, F:] = 0
y604 = torch.empty(v1, 608, device=dev)
us_gp4 = t(lambda: ctx.spmm_csc_fwd(l1.column_offset, l1.row_indices, l1.edge_weight_forward,
                                    l1.sizes[0:1], v1, featp4[:, :604], y604[:, :604], row_map=l1.source))
print(f"  same, 604 columns as float4: {us_gp4:.1f} us")
Hm = torch.randn(s1, 128, device=dev)
y128 = torch.empty(v1, 128, device=dev)
us_a = t(lambda: ctx.spmm_csc_fwd(l1.column_offset, l1.row_indices, l1.edge_weight_forward,
                                  l1.sizes[0:1], v1, Hm, y128))
print(f"agg 128 fwd: {us_a:.1f} us")
gz = torch.randn(v1, 128, device=dev)
gi = torch.empty(s1, 128, device=dev)
us_b = t(lambda: ctx.spmm_csr_bwd(l1.row_offset, l1.column_indices, l1.edge_weight_backward,
                                  l1.sizes[2:3], s1, gz, gi))
print(f"agg 128 bwd (CSR): {us_b:.1f} us")
W = torch.randn(F, 128, device=dev)
Z = torch.empty(v1, 128, device=dev)
us_nn = t(lambda: ctx.gemm(y602, W, Z))
X0 = feat[l1.source[:s1].long()]
Hx = torch.empty(s1, 128, device=dev)
us_nn2 = t(lambda: ctx.gemm(X0, W, Hx))
D = torch.empty(F, 128, device=dev)
us_tn = t(lambda: ctx.gemm(y602, gz, D, trans_a=True))
gi2 = torch.randn(s1, 128, device=dev)
us_tn2 = t(lambda: ctx.gemm(X0, gi2, D, trans_a=True))
print(f"ref order : agg602 {us_g:.0f} + NN[{v1}] {us_nn:.0f} + TN[{v1}] {us_tn:.0f} = {us_g + us_nn + us_tn:.0f} us")
print(f"transform : NN[{s1}] {us_nn2:.0f} + agg128 {us_a:.0f} + bwd128 {us_b:.0f} + TN[{s1}] {us_tn2:.0f} = "
      f"{us_nn2 + us_a + us_b + us_tn2:.0f} us (+ CSR build {us_s_csr - us_s:.0f} us on the sampler stream)")
