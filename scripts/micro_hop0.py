"""Hop-0 post-mask CSR backward at C2 (the hop above the transform-first
bottom layer): its row-length profile and time, against the same gather with
every row cut to its first 32 edges (no hub rows for the block-cooperative
path) — how much of the kernel is the hubs' tail.

  python scripts/micro_hop0.py [--iters 20]
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "sample-based-gnn_amd"))
sys.path.insert(0, str(ROOT / "scripts"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from micro_agg import timeit  # noqa: E402


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
    l = lay[0]
    v, e, s = l["v_size"], l["e_size"], l["src_size"]
    ro = l["row_offset"][: s + 1].to(torch.int64)
    ln = ro[1:] - ro[:-1]
    q = torch.quantile(ln.double(), torch.tensor([0.5, 0.9, 0.99, 0.999], dtype=torch.float64, device=dev))
    long = ln > 32
    out = {"v": v, "e": e, "s": s, "len_q50_90_99_999": [round(float(x), 1) for x in q],
           "len_max": int(ln.max()), "rows_gt32": int(long.sum()),
           "edges_in_rows_gt32": int(ln[long].sum())}
    gen = torch.Generator(device=dev).manual_seed(3)
    dZ = torch.randn(v, 128, device=dev, generator=gen)
    Xa = torch.relu(torch.randn(s, 128, device=dev, generator=gen))
    dH = torch.empty(s, 128, device=dev)
    sdev = torch.tensor([s], dtype=torch.int32, device=dev)
    ci, wb = l["column_indices"], l["edge_weight_backward"]
    out["postmask_us"] = round(timeit(lambda: hip.spmm_csr_bwd_postmask(
        l["row_offset"], ci, wb, sdev, s, dZ, Xa, dH, scale=2.0), a.iters), 1)
    out["plain_us"] = round(timeit(lambda: hip.spmm_csr_bwd(
        l["row_offset"], ci, wb, sdev, s, dZ, dH), a.iters), 1)
    # every row cut to its first 32 edges
    lc = torch.clamp(ln, max=32)
    ro2 = torch.zeros(s + 1, dtype=torch.int64, device=dev)
    ro2[1:] = torch.cumsum(lc, 0)
    pos = torch.repeat_interleave(ro[:-1], lc) + (torch.arange(int(ro2[-1]), device=dev) -
                                                  torch.repeat_interleave(ro2[:-1], lc))
    ci2, wb2 = ci[pos].contiguous(), wb[pos].contiguous()
    ro2 = ro2.to(torch.int32)
    out["postmask_cut32_us"] = round(timeit(lambda: hip.spmm_csr_bwd_postmask(
        ro2, ci2, wb2, sdev, s, dZ, Xa, dH, scale=2.0), a.iters), 1)
    out["e_cut32"] = int(ro2[-1])
    # the mask read + output write alone (no edges)
    ro3 = torch.zeros(s + 1, dtype=torch.int32, device=dev)
    out["postmask_no_edges_us"] = round(timeit(lambda: hip.spmm_csr_bwd_postmask(
        ro3, ci2, wb2, sdev, s, dZ, Xa, dH, scale=2.0), a.iters), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
