"""Does a captured HIP graph shorten the sampler chain on the GPU?  Three-layer
products-shaped sampling (B=1024, fanout 15-10-5, CSR on the two upper
layers): direct launches vs one graph replay.  GPU box only."""
import pathlib
import sys
import time

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1] / "sample-based-gnn_amd"))
import torch  # noqa: E402

from nts import hip as H, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
shape = sys.argv[1] if len(sys.argv) > 1 else "products"
fan = [15, 10, 5] if shape == "products" else [25, 10]
B = 1024 if shape == "products" else 10000
g, F, C = synthetic.shaped(shape, device=dev)
s = torch.cuda.Stream(device=dev)
ctx = H.HipContext(0, stream=s, seed=2000)
with torch.cuda.stream(s):
    col, rows = ctx.build_csc(g.src, g.dst, g.n_vertices)
    od, idg = ctx.degrees(g.src, g.dst, g.n_vertices)
G = H.DeviceGraph(g.n_vertices, g.n_edges, col, rows, idg, od)
seeds = torch.randperm(g.n_vertices, device=dev)[:B].to(torch.int32)
caps = H.layer_caps(B, fan, g.n_vertices, g.n_edges)
ctx.reserve(g.n_vertices, max(max(c) for c in caps))
vsz = torch.tensor([B], dtype=torch.int32, device=dev)
torch.cuda.synchronize()
layers = []
cur, cv = seeds, vsz
for l, (f, c) in enumerate(zip(fan, caps)):
    lay = H.LayerBuffers(*c, cur, cv, dev, csr=l < len(fan) - 1)
    layers.append(lay)
    cur, cv = lay.source, lay.sizes[2:3]


def run():
    for l, (f, lay) in enumerate(zip(fan, layers)):
        ctx.sample_layer(G, lay, f, l, 0, 0, 0)


with torch.cuda.stream(s):
    for _ in range(5):
        run()
torch.cuda.synchronize()


def t(fn, it=50):
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        a.record()
        h0 = time.perf_counter()
        for _ in range(it):
            fn()
        h1 = time.perf_counter()
        b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3, (h1 - h0) / it * 1e6


us, host = t(run)
print(f"[{shape}] direct: {us:.1f} us/batch GPU, host issue {host:.1f} us", flush=True)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr, stream=s):
    run()
torch.cuda.synchronize()
us2, host2 = t(gr.replay)
print(f"[{shape}] graph : {us2:.1f} us/batch GPU, host issue {host2:.1f} us", flush=True)
print("sizes", [l.sizes_host() for l in layers])
