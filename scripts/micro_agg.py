"""Micro benchmark of the transform-first bottom layer's aggregations at C2
size, alone on the GPU: the forward A H with relu/dropout (spmm_csc_fwd_act)
and the backward A^T dZ with rs-scaled column maxima (spmm_csr_bwd_colmax),
plus the hop-0 forward / post-mask backward — time per call and the rate of
the gathered rows (every edge's 512-byte row) and of the algorithmic bytes.

  python scripts/micro_agg.py [--iters 20]   (NTS_HIP_LIB=scripts/probe/lib_agglds/libnts_hip.so: the k_agg_lds variant, make variant V=agglds VFLAGS=-DNTS_WITH_AGG_LDS)
"""
import argparse
import json
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sample-based-gnn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from nts import host, synthetic
    from nts.hip import HipContext
    E = host.ext()
    dev = torch.device("cuda:0")
    g, F, C = synthetic.shaped("reddit", device=dev)
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    B = 10_000
    seeds = torch.from_numpy(np.random.default_rng(5).choice(V, B, replace=False).astype(np.int32))
    lay = E.FastSampler(G, seeds, 2, B, [25, 10]).sample_gpu_fast(B)
    hip = HipContext(0)
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith("NTS_")}}
    gen = torch.Generator(device=dev).manual_seed(3)
    for name, l in (("bottom", lay[1]), ("hop0", lay[0])):
        v, e, s = l["v_size"], l["e_size"], l["src_size"]
        H = torch.randn(s, 128, device=dev, generator=gen)
        Y = torch.empty(v, 128, device=dev)
        fwd = timeit(lambda: hip.spmm_csc_fwd_act(l["column_offset"], l["row_indices"],
                                                  l["edge_weight_forward"], None, v, H, Y, p=0.5,
                                                  seed=7, offset=1), a.iters)
        dZ = torch.randn(v, 128, device=dev, generator=gen)
        dH = torch.empty(s, 128, device=dev)
        if name == "bottom":
            R = hip.colmax_rows_per_part(128)
            parts = torch.empty((s + R - 1) // R, 128, dtype=torch.int32, device=dev)
            rs = torch.ones(V, device=dev)
            bwd = timeit(lambda: hip.spmm_csr_bwd_colmax(l["row_offset"], l["column_indices"],
                                                         l["edge_weight_backward"], None, s, dZ, dH,
                                                         parts, rs=rs, rows=l["source"]), a.iters)
        else:
            Xa = torch.relu(torch.randn(s, 128, device=dev, generator=gen))
            bwd = timeit(lambda: hip.spmm_csr_bwd_postmask(l["row_offset"], l["column_indices"],
                                                           l["edge_weight_backward"], None, s, dZ, Xa,
                                                           dH, scale=2.0), a.iters)
        alg_f = 512.0 * s + 8.0 * e + 4.0 * (v + 1) + 512.0 * v
        alg_b = 512.0 * v + 8.0 * e + 4.0 * (s + 1) + 512.0 * s
        out[name] = {"v": v, "e": e, "s": s, "fwd_us": round(fwd, 1), "bwd_us": round(bwd, 1),
                     "fwd_rows_TBps": round(512.0 * e / fwd / 1e6, 2),
                     "bwd_rows_TBps": round(512.0 * e / bwd / 1e6, 2),
                     "fwd_alg_frac": round(alg_f / fwd / 1e6 / 8.0, 3),
                     "bwd_alg_frac": round(alg_b / bwd / 1e6 / 8.0, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
