"""Source-row reuse of the C2 bottom-layer aggregation:
one Reddit-shaped batch (B = 10,000, 25-10, the bench's sampler, Philox) —
how the ~1.36 M gathered rows of H (512 B each) spread over the ~229 K
distinct source rows, how much of the edge traffic the hottest rows carry,
and what a dst-range split over the 8 XCDs (each L2 4 MiB = 8,192 H rows)
would leave per XCD.

  python scripts/reuse_probe.py   (GPU: samples with the product sampler)
"""
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sample-based-gnn_amd"))

import torch  # noqa: E402

from nts import host, synthetic  # noqa: E402


def main():
    E = host.ext()
    g, F, C = synthetic.shaped("reddit", device="cuda:0")
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    B, fan = 10_000, [25, 10]
    seeds = torch.from_numpy(np.random.default_rng(5).choice(V, B, replace=False).astype(np.int32))
    fs = E.FastSampler(G, seeds, 2, B, fan)
    layers = fs.sample_gpu_fast(B)
    bot = layers[1]  # the bottom layer: dsts = hop-1 frontier, srcs = the H rows gathered
    v, e, s = int(bot["v_size"]), int(bot["e_size"]), int(bot["src_size"])
    ri = bot["row_indices"][:e].cpu().numpy().view(np.uint32).astype(np.int64)  # local src per edge
    co = bot["column_offset"][:v + 1].cpu().numpy().view(np.uint32).astype(np.int64)
    cnt = np.bincount(ri, minlength=s)
    order = np.sort(cnt)[::-1]
    cum = np.cumsum(order)
    out = {"dsts": v, "edges": e, "distinct_srcs": s, "edges_per_src_mean": e / s,
           "max_src_reuse": int(order[0])}
    for k in (256, 1024, 4096, 8192, 16384, 65536):
        out[f"edge_share_top{k}"] = float(cum[min(k, s) - 1] / e)
    hist = {str(b): int(((cnt >= lo) & (cnt < hi)).sum())
            for b, (lo, hi) in {"1": (1, 2), "2-3": (2, 4), "4-7": (4, 8), "8-15": (8, 16),
                                "16-63": (16, 64), ">=64": (64, 1 << 40)}.items()}
    out["srcs_by_reuse"] = hist
    # dst range split into 8 contiguous parts (one per XCD): distinct srcs per
    # part and the share of a part's edges its own top-8192 rows carry
    parts = []
    for p in range(8):
        d0, d1 = v * p // 8, v * (p + 1) // 8
        r = ri[co[d0]:co[d1]]
        c = np.bincount(r, minlength=s)
        nz = np.sort(c[c > 0])[::-1]
        parts.append({"edges": int(r.size), "distinct_srcs": int(nz.size),
                      "top8192_share": float(nz[:8192].sum() / max(r.size, 1))})
    out["per_xcd_dst_range"] = parts
    out["re_reads_per_row"] = e / s
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
