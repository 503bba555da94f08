"""Full-size correctness of the benched configurations.

The parity suite runs on Cora-sized graphs; these tests run the HIP path at
the sizes BASELINE.json's configs are benched on and check it there:
  * C2 Reddit-shaped (V=232,965, E~114.8M, batch 10,000, fanout 25-10): the
    whole sampled batch bit-exact vs the oracle's PHILOX restatement of
    FastSampler::sample_fast (core/ntsFastSampler.hpp:962-1140), the fused
    gather + hop-1 aggregation bit-exact vs MiniBatchFuseOp, the
    transform-first bottom layer within 1e-4 of the GCN_CPU_SAMPLE chain, and
    the size-independent properties (source strictly ascending, row_indices <
    src_size, e_size = sum min(deg, f), sampled ids a sub-multiset of each
    dst's neighbour list).
  * C3 ogbn-products-shaped, 3 layers 15-10-5, batch 1,024, Mean weights:
    the same sampler checks and the bottom aggregation.
  * C5-class: a graph past 2^31 edges (u64 CSC offsets, the sampler reading
    neighbour lists that start beyond 2^31) and a feature table past 2^32
    floats (64-bit row offsets in the gathers).
Memory is freed between tests; each runs in well under the per-test limit.
"""
import gc

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def E():
    from nts import host
    return host.ext()


def _np(t):
    a = t.cpu().numpy()
    return a.view(np.uint32) if a.dtype == np.int32 else a


def _free():
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _properties(G, layers, fanout, V):
    """Size-independent properties of one sampled batch, on the device."""
    col = G.column_offset  # int64 [V+1]
    rows = G.row_indices.long() & 0xFFFFFFFF
    for ly, f in zip(layers, fanout):
        v, e, s = ly["v_size"], ly["e_size"], ly["src_size"]
        dst = ly["destination"].long() & 0xFFFFFFFF
        src = ly["source"].long() & 0xFFFFFFFF
        co = ly["column_offset"].long()
        ri = ly["row_indices"].long() & 0xFFFFFFFF
        ans = ly["sample_ans"].long() & 0xFFFFFFFF
        deg = col[dst + 1] - col[dst]
        want = deg if f < 0 else torch.clamp(deg, max=f)
        assert int(want.sum()) == e, "e_size != sum min(deg, f)"
        assert torch.equal(co[1:] - co[:-1], want), "per-dst counts"
        assert bool((src[1:] > src[:-1]).all()), "source not strictly ascending"
        assert int(src.max()) < V
        assert bool((ri < s).all()), "row_indices >= src_size"
        assert torch.equal(src[ri], ans), "row_indices do not map to sample_ans"
        # every sampled id is a neighbour of its dst, at most as often as it
        # occurs in the neighbour list (distinct positions of a multigraph)
        d_of_e = torch.repeat_interleave(torch.arange(v, device=DEV), want)
        ks = torch.sort(d_of_e * V + ans).values
        uk, cnt = torch.unique_consecutive(ks, return_counts=True)
        n_of = torch.repeat_interleave(torch.arange(v, device=DEV), deg)
        base = torch.repeat_interleave(col[dst] - torch.cumsum(deg, 0) + deg, deg)
        nbr = rows[base + torch.arange(int(deg.sum()), device=DEV)]
        kn = torch.sort(n_of * V + nbr).values
        have = torch.searchsorted(kn, uk, right=True) - torch.searchsorted(kn, uk, right=False)
        assert bool((have >= cnt).all()), "a sampled id is not a neighbour (or repeats a position)"
        del ks, uk, cnt, n_of, base, nbr, kn, have, d_of_e


def _compare_oracle(got, ref):
    for a, b in zip(got, ref):
        assert (a["v_size"], a["e_size"], a["src_size"]) == (b["v_size"], b["e_size"], b["src_size"])
        for k in ("destination", "column_offset", "row_indices", "sample_ans", "source",
                  "edge_weight_forward", "row_offset", "column_indices", "edge_weight_backward"):
            if k in a and a[k] is not None:
                assert np.array_equal(_np(a[k]), b[k]), k


def test_c2_reddit_shaped_full_batch(E):
    from nts import host, synthetic
    g, F, C = synthetic.shaped("reddit", device=DEV)
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    src_h, dst_h = g.src.cpu().numpy().view(np.uint32), g.dst.cpu().numpy().view(np.uint32)
    del g
    fan, B = [25, 10], 10_000
    seeds = torch.from_numpy(np.random.default_rng(5).choice(V, B, replace=False).astype(np.int32))
    fs = E.FastSampler(G, seeds, 2, B, fan)
    got = fs.sample_gpu_fast(B)
    _properties(G, got, fan, V)
    assert got[1]["e_size"] > 1_000_000 and got[1]["src_size"] > 200_000  # the benched shape
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    od, idg = orc.degrees(V, src_h, dst_h)
    assert np.array_equal(od, _np(G.out_degree)) and np.array_equal(idg, _np(G.in_degree))
    o = orc.Sampler(col, rows, idg, od, fan, rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    ref = o.sample(seeds.numpy().astype(np.uint32), 0)
    _compare_oracle(got, ref)
    # fused gather + hop-1 aggregation (the bottom graph op) bit-exact, full batch
    from nts.hip import HipContext
    hip = HipContext(0)
    feat = synthetic.features(V, F, device=DEV)
    l1 = got[1]
    v1 = l1["v_size"]
    y = torch.empty(v1, F, device=DEV)
    hip.spmm_csc_fwd(l1["column_offset"], l1["row_indices"], l1["edge_weight_forward"], None, v1,
                     feat, y, row_map=l1["source"])
    X0 = orc.get_feature(ref[1]["source"], feat.cpu().numpy(), threads=8)
    Y0 = orc.fuse_fwd(ref[1], X0, od, idg, threads=8)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), Y0)
    # transform-first bottom layer at full size: A (X W) vs (A X) W within 1e-4
    W = torch.randn(F, 128, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1)) * 0.05
    H = torch.empty(l1["src_size"], 128, device=DEV)
    hip.gemm_gather(feat, l1["source"], W, H)
    X1 = torch.empty(v1, 128, device=DEV)
    hip.spmm_csc_fwd_act(l1["column_offset"], l1["row_indices"], l1["edge_weight_forward"], None,
                         v1, H, X1, p=0.0)
    ref_x1 = torch.relu(torch.from_numpy(Y0).to(DEV).double() @ W.double())
    torch.testing.assert_close(X1.double(), ref_x1, rtol=1e-4, atol=1e-4)
    # the benched arithmetic: the same layer on the f16 pair table (planar), and
    # its weight gradient X[src]^T dH, at full size (src ~229 K rows)
    Q, rs = hip.h2_split_rows_planar(feat)
    H2 = torch.empty_like(H)
    hip.gemm_h2p_gather(Q, rs, l1["source"], W, H2)
    X1b = torch.empty_like(X1)
    hip.spmm_csc_fwd_act(l1["column_offset"], l1["row_indices"], l1["edge_weight_forward"], None,
                         v1, H2, X1b, p=0.0)
    torch.testing.assert_close(X1b.double(), ref_x1, rtol=1e-4, atol=1e-4)
    gH = torch.randn(l1["src_size"], 128, device=DEV,
                     generator=torch.Generator(device=DEV).manual_seed(2)) * 1e-4
    dW = torch.full((F, 128), float("nan"), device=DEV)
    hip.gemm_h2p_tn_gather(Q, rs, l1["source"], gH, dW, F)
    Xs = feat[l1["source"].long()].double()
    ref_dw = Xs.t() @ gH.double()
    nerr = ((dW.double() - ref_dw).abs() / (Xs.abs().t() @ gH.double().abs() + 1e-300)).max().item()
    assert nerr < 1e-6, nerr
    del fs, got, feat, y, H, X1, G, Q, rs, H2, X1b, gH, dW, Xs, ref_dw
    _free()


def test_fresh_context_frontier_past_resident_tiles(E):
    """Regression for the C5 hang: a fresh sampler context whose
    first layer grows the look-back tile states right before a frontier
    compaction of more tiles than the chip holds at once (V = 24 M: 5,860
    tiles of 4,096 vertices).  The states were zeroed on the NULL stream,
    unordered with the sampler's stream.  Three batches, every array
    bit-exact vs the oracle's PHILOX restatement of sample_fast
    (core/ntsFastSampler.hpp:962-1140)."""
    V, Ecount, B, fan = 24_000_000, 48_000_000, 4096, [10, 5]
    gen = torch.Generator(device=DEV).manual_seed(11)
    src = torch.randint(0, V, (Ecount,), device=DEV, generator=gen, dtype=torch.int32)
    dst = torch.randint(0, V, (Ecount,), device=DEV, generator=gen, dtype=torch.int32)
    G = E.FullyRepGraph.from_edges(src, dst, V)
    del src, dst
    _free()
    seeds = torch.from_numpy(np.random.default_rng(7).choice(V, 3 * B, replace=False).astype(np.int32))
    fs = E.FastSampler(G, seeds, 2, B, fan)
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    o = orc.Sampler(col, rows, _np(G.in_degree), _np(G.out_degree), fan, rng_mode=orc.RNG_PHILOX,
                    order_mode=orc.ORDER_DRAW)
    for b in range(3):
        got = fs.sample_gpu_fast(B)
        assert got[1]["src_size"] > 10_000  # random ids: the frontier spans the whole vertex range
        ref = o.sample(seeds.numpy()[b * B:(b + 1) * B].astype(np.uint32), b)
        _compare_oracle(got, ref)
    del fs, got, G, o
    _free()


def _sets_equal(got_layer, ref_layer):
    """Per-dst neighbour multisets equal (the reference emits std::unordered_map
    order inside a dst, core/ntsFastSampler.hpp:1026-1038)."""
    co = _np(got_layer["column_offset"]).astype(np.int64)
    d_of_e = np.repeat(np.arange(co.size - 1, dtype=np.int64), np.diff(co))
    a = _np(got_layer["sample_ans"]).astype(np.int64)
    b = ref_layer["sample_ans"].astype(np.int64)
    ka = np.sort(d_of_e * (1 << 32) + a)
    kb = np.sort(d_of_e * (1 << 32) + b)
    return np.array_equal(ka, kb)


def test_c2_mt19937_reference_stream_full_batch(E):
    """The reference's own generator at the benched size: std::mt19937(2000) +
    uniform_int_distribution (Lemire, libstdc++ 11) consumed over the dsts in
    order (core/ntsFastSampler.hpp:200-205,962-1140).  Two consecutive C2
    batches (B=10,000, 25-10): every array bit-exact vs the oracle in draw
    order, per-dst sets equal to the reference's unordered_map order, and the
    generator state (624 words + position) identical after each batch."""
    from nts import synthetic
    g, F, C = synthetic.shaped("reddit", device=DEV)
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    fan, B = [25, 10], 10_000
    rng = np.random.default_rng(15)
    perm = rng.permutation(V).astype(np.int32)[:2 * B]
    fs = E.FastSampler(G, torch.from_numpy(perm), 2, B, fan, rng_mode=1, seed=2000)
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    od, idg = _np(G.out_degree), _np(G.in_degree)
    o = orc.Sampler(col, rows, idg, od, fan, seed=2000, rng_mode=orc.RNG_MT_LEMIRE,
                    order_mode=orc.ORDER_DRAW)
    o_map = orc.Sampler(col, rows, idg, od, fan, seed=2000, rng_mode=orc.RNG_MT_LEMIRE,
                        order_mode=orc.ORDER_UNORDERED_MAP)
    for b in range(2):
        got = fs.sample_gpu_fast(B)
        _properties(G, got, fan, V)
        assert got[1]["e_size"] > 1_000_000
        seeds = perm[b * B:(b + 1) * B].view(np.uint32)
        ref = o.sample(seeds, b)
        _compare_oracle(got, ref)
        assert np.array_equal(_np(fs.rng_state()), o.mt_state()), f"generator state, batch {b}"
        ref_map = o_map.sample(seeds, b)
        for a, r in zip(got, ref_map):
            assert np.array_equal(_np(a["source"]), r["source"])
            assert _sets_equal(a, r)
    del fs, got, G
    _free()


def test_c2_mt19937_short_stream_reruns(E):
    """A layer whose MT19937 draws outrun the words generated for it is not
    fatal: the first bounds are forced 20x too small
    (nts_hip_mt_budget_scale), three C2 batches (B = 10,000, 25-10) are issued
    into three slots ahead of the first finish — the pipelined driver's order
    — and finishing the first one rewinds the generator to its checkpoint,
    raises the bounds and samples it and the two behind it again.  Every batch
    (and two more, sampled synchronously) bit-exact vs the oracle's
    std::mt19937(2000) walk, and the generator state identical after the
    last: the re-runs read the same stream (core/ntsFastSampler.hpp:200-205,
    962-1140)."""
    from nts import synthetic
    g, F, C = synthetic.shaped("reddit", device=DEV)
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    fan, B, nb = [25, 10], 10_000, 5
    rng = np.random.default_rng(21)
    perm = rng.permutation(V).astype(np.int32)[:nb * B]
    fs = E.FastSampler(G, torch.from_numpy(perm), 2, B, fan, rng_mode=1, seed=2000, pipeline=3)
    fs.set_mt_budget_scale(0.05)
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    o = orc.Sampler(col, rows, _np(G.in_degree), _np(G.out_degree), fan, seed=2000,
                    rng_mode=orc.RNG_MT_LEMIRE, order_mode=orc.ORDER_DRAW)
    for slot in range(3):
        fs.issue(B, slot)
    for b in range(nb):
        if b < 3:
            got = fs.finish(b)
        else:
            fs.issue(B, b % 3)
            got = fs.finish(b % 3)
        _compare_oracle(got, o.sample(perm[b * B:(b + 1) * B].view(np.uint32), b))
        if b == 0:
            assert fs.mt_reruns >= 1 and fs.mt_budget_scale > 0.05, (fs.mt_reruns, fs.mt_budget_scale)
    assert np.array_equal(_np(fs.rng_state()), o.mt_state())
    del fs, got, G
    _free()


def test_c2_mt19937_stream_ring_wraps(E):
    """The MT19937 stream ring (2^25 tempered words on the device, generated
    ahead of the layers that read them) wrapping around: 24 consecutive C2
    batches (B = 10,000, 25-10) consume more than 2^25 words, so the later
    layers read words stored at ring index (stream word mod 2^25) and the
    generator refills slots that earlier layers read — the host-side
    bookkeeping (read-back position, pending bounds, the ring-capacity wait in
    mt_ring_prepare) included.  Every batch bit-exact vs the oracle's
    std::mt19937(2000) walk in draw order (core/ntsFastSampler.hpp:200-205,
    962-1140), the generator state identical after the last."""
    from nts import synthetic
    g, F, C = synthetic.shaped("reddit", device=DEV)
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    fan, B, nb = [25, 10], 10_000, 24
    rng = np.random.default_rng(17)
    perm = np.concatenate([rng.permutation(V), rng.permutation(V)]).astype(np.int32)[:nb * B]
    fs = E.FastSampler(G, torch.from_numpy(perm), 2, B, fan, rng_mode=1, seed=2000)
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    o = orc.Sampler(col, rows, _np(G.in_degree), _np(G.out_degree), fan, seed=2000,
                    rng_mode=orc.RNG_MT_LEMIRE, order_mode=orc.ORDER_DRAW)
    edges = 0
    for b in range(nb):
        got = fs.sample_gpu_fast(B)
        edges += sum(int(l["e_size"]) for l in got)
        ref = o.sample(perm[b * B:(b + 1) * B].view(np.uint32), b)
        _compare_oracle(got, ref)
    assert edges > (1 << 25), edges  # at least one accepted word per edge: the ring wrapped
    assert np.array_equal(_np(fs.rng_state()), o.mt_state())
    del fs, got, G
    _free()


def test_c3_products_shaped_three_layers_mean(E):
    from nts import synthetic
    g, F, C = synthetic.shaped("products", device=DEV)
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    fan, B = [15, 10, 5], 1024
    seeds = torch.from_numpy(np.random.default_rng(6).choice(V, B, replace=False).astype(np.int32))
    fs = E.FastSampler(G, seeds, 3, B, fan)
    got = fs.sample_gpu_fast(B, E.WeightType.Mean)
    _properties(G, got, fan, V)
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    od, idg = _np(G.out_degree), _np(G.in_degree)
    o = orc.Sampler(col, rows, idg, od, fan, rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    ref = o.sample(seeds.numpy().astype(np.uint32), 0, orc.W_MEAN)
    _compare_oracle(got, ref)
    from nts.hip import HipContext
    hip = HipContext(0)
    feat = synthetic.features(V, F, device=DEV)
    l2 = got[2]
    y = torch.empty(l2["v_size"], F, device=DEV)
    hip.spmm_csc_fwd(l2["column_offset"], l2["row_indices"], l2["edge_weight_forward"], None,
                     l2["v_size"], feat, y, row_map=l2["source"])
    X0 = orc.get_feature(ref[2]["source"], feat.cpu().numpy(), threads=8)
    Y0 = orc.fuse_fwd(ref[2], X0, od, idg, weight_mean=True, threads=8)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), Y0)
    del fs, got, feat, y, G
    _free()


def test_c3_mt19937_three_layers(E):
    """C3's sampling (products-shaped, 15-10-5, batch 1,024) on the
    reference's own generator stream: every array of the three layers
    bit-exact vs the oracle's std::mt19937(2000) walk in draw order and the
    generator state identical after each of two batches."""
    from nts import synthetic
    g, F, C = synthetic.shaped("products", device=DEV)
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    fan, B = [15, 10, 5], 1024
    perm = np.random.default_rng(16).permutation(V).astype(np.int32)[:2 * B]
    fs = E.FastSampler(G, torch.from_numpy(perm), 3, B, fan, rng_mode=1, seed=2000)
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    od, idg = _np(G.out_degree), _np(G.in_degree)
    o = orc.Sampler(col, rows, idg, od, fan, seed=2000, rng_mode=orc.RNG_MT_LEMIRE,
                    order_mode=orc.ORDER_DRAW)
    for b in range(2):
        got = fs.sample_gpu_fast(B, E.WeightType.Mean)
        _properties(G, got, fan, V)
        ref = o.sample(perm[b * B:(b + 1) * B].view(np.uint32), b, orc.W_MEAN)
        _compare_oracle(got, ref)
        assert np.array_equal(_np(fs.rng_state()), o.mt_state()), f"generator state, batch {b}"
    del fs, got, G
    _free()


def test_c4_products_shaped_two_layer_gcn(E):
    """C4's per-GPU workload (GCN_SAMPLE_ALL_MULTI, products-shaped, 100-256-47,
    fanout 25-10, B=1,024 per GPU): the sampled batch bit-exact vs the
    oracle's PHILOX restatement, with the size-independent properties, and the
    bottom aggregation (fused gather) bit-exact vs MiniBatchFuseOp."""
    from nts import synthetic
    from nts.hip import HipContext
    g, F, C = synthetic.shaped("products", device=DEV)
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    fan, B = [25, 10], 1024
    seeds = torch.from_numpy(np.random.default_rng(44).choice(V, B, replace=False).astype(np.int32))
    fs = E.FastSampler(G, seeds, 2, B, fan)
    got = fs.sample_gpu_fast(B)
    _properties(G, got, fan, V)
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    od, idg = _np(G.out_degree), _np(G.in_degree)
    o = orc.Sampler(col, rows, idg, od, fan, rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    ref = o.sample(seeds.numpy().astype(np.uint32), 0)
    _compare_oracle(got, ref)
    hip = HipContext(0)
    feat = synthetic.features(V, F, device=DEV)
    l1 = got[1]
    y = torch.empty(l1["v_size"], F, device=DEV)
    hip.spmm_csc_fwd(l1["column_offset"], l1["row_indices"], l1["edge_weight_forward"], None,
                     l1["v_size"], feat, y, row_map=l1["source"])
    Y0 = orc.fuse_fwd(ref[1], orc.get_feature(ref[1]["source"], feat.cpu().numpy(), threads=8),
                      od, idg, threads=8)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), Y0)
    del fs, got, feat, y, G
    _free()


def test_c5_papers_shaped_pd_cache_with_feature_spill(E):
    """C5 as BASELINE.json states it, at one GPU: GS_SAMPLE_PD_CACHE
    (toolkits/GS_SAMPLE_PD_CACHE.hpp:673-1112) on the papers100M-shaped graph
    (V=111 M, E=3.34 B, 128-wide features, 128-256-256-172, 15-10-5, B=1,024,
    GraphSAGE mean weights), the feature table in pinned host memory with 30 %
    of its rows (highest degree) cached in HBM, and the NeutronOrch PD cache
    (hot vertices of each super-batch of 4 batches, rate 0.2).  The training
    seeds are the first 8 batches' worth: preSample over all 17.6 K
    super-batches would keep ~10^10 hot ids (the reference allocates
    cache_rate * V * super_batches of them, core/ntsBaseOp.hpp:424).
    Checked at full size: super-batch 0's hot set == the oracle's
    get_most_neighbor; the first trained batch == the oracle sampler with
    those dsts omitted (every array, bit-exact; sample_gpu_fast_omit,
    core/ntsFastSampler.hpp:711-915); no capacity overflow; source strictly
    ascending; every sampled id a real neighbour; and finite training."""
    from nts import host, synthetic
    g, F, C = synthetic.shaped("papers100m", device=DEV)
    V = g.n_vertices
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    _free()
    fan, B, sb = [15, 10, 5], 1024, 4
    rng = np.random.default_rng(55)
    train = torch.from_numpy(rng.choice(V, 8 * B, replace=False).astype(np.int32))
    feat = synthetic.features(V, F, device=DEV)
    labels = torch.randint(0, C, (V,), device=DEV, generator=torch.Generator(device=DEV).manual_seed(5))
    cfg = host.gcn_config([F, 256, 256, C], fan, B, weight="mean", learn_rate=0.01, drop_rate=0.0,
                          shuffle=False, pd_cache=True, pd_rate=0.2, pd_super_batch=sb,
                          cache_rate=0.3)
    drv = E.GCN_SAMPLE_ALLGPU_impl(G, feat, labels, train, cfg)
    del feat
    _free()
    counts, ids = drv.presample()
    assert len(counts) == 2
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    t = train.numpy().astype(np.uint32)
    _, hot_ref = orc.presample(col, rows, t[:sb * B], len(fan), 0.2)
    hot = np.array(ids[:counts[0]], np.uint32)
    assert np.array_equal(hot, hot_ref) and hot.size > 1000
    drv.train_batch()
    drv.synchronize()
    assert torch.isfinite(drv.loss).item()
    got = drv.last_layers
    # the first batch: the bottom layer sampled with super-batch 0's hot dsts omitted
    od, idg = _np(G.out_degree), _np(G.in_degree)
    omap = np.full(V, 0xFFFFFFFF, np.uint32)
    omap[hot] = 1
    o = orc.Sampler(col, rows, idg, od, fan, rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    o.set_omit(omap, 1)
    ref = o.sample(t[:B], 0, orc.W_MEAN)
    _compare_oracle(got, ref)
    bottom = ref[-1]
    cnt = np.diff(bottom["column_offset"].astype(np.int64))
    om = np.isin(bottom["destination"], hot)
    assert om.sum() > 100 and (cnt[om] == 0).all()
    for ly in got:
        src = ly["source"].long() & 0xFFFFFFFF
        assert bool((src[1:] > src[:-1]).all())
        assert bool(((ly["row_indices"].long() & 0xFFFFFFFF) < ly["src_size"]).all())
    # every sampled id of the top two layers is a real neighbour (distinct positions)
    _properties(G, got[:2], fan[:2], V)
    for _ in range(5):  # through super-batch 1 (new hot set, shared embedding re-made)
        drv.train_batch()
    drv.synchronize()
    assert torch.isfinite(drv.loss).item()
    del drv, got, G, rows, col
    _free()


def test_c5_class_past_2e31_edges(E):
    """u64 CSC offsets: 2.3 x 10^9 edges on 2M vertices; seeds whose neighbour
    lists start past 2^31 are sampled bit-exactly vs the oracle."""
    from nts import synthetic
    V, En = 2_000_000, 2_300_000_000
    g = synthetic.chung_lu(V, En, 20.0, device=DEV, seed=77)
    G = E.FullyRepGraph.from_edges(g.src, g.dst, V)
    del g
    _free()
    col_d = G.column_offset
    assert int(col_d[-1]) == En and int(col_d[-1]) > 2 ** 31
    late = torch.nonzero(col_d[:-1] > 2 ** 31 + 5).flatten()
    seeds = late[torch.randperm(late.numel(), device=DEV,
                                generator=torch.Generator(device=DEV).manual_seed(3))[:512]]
    seeds = seeds.to(torch.int32).cpu()
    fan = [15, 10]
    fs = E.FastSampler(G, seeds, 2, 512, fan)
    got = fs.sample_gpu_fast(512)
    _properties(G, got, fan, V)
    col = col_d.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    od, idg = _np(G.out_degree), _np(G.in_degree)
    o = orc.Sampler(col, rows, idg, od, fan, rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    ref = o.sample(seeds.numpy().astype(np.uint32), 0)
    _compare_oracle(got, ref)
    del fs, got, G, rows
    _free()


def test_feature_rows_past_2e32_floats(E):
    """64-bit row offsets in the gathers: a [35M x 128] fp32 table (4.48 x 10^9
    floats, 17.9 GB); rows past the 2^32-float mark are gathered, aggregated
    and multiplied (row-gathered GEMM) exactly like torch indexing of them."""
    from nts.hip import HipContext
    hip = HipContext(0)
    Vt, F = 35_000_000, 128
    table = torch.empty(Vt, F, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(9)
    ids = torch.randint(2 ** 32 // F + 1, Vt, (4096,), device=DEV, generator=gen)
    ids[:16] = torch.arange(Vt - 16, Vt, device=DEV)
    table[ids] = torch.randn(ids.numel(), F, device=DEV, generator=gen)
    idx = ids.to(torch.int32)
    n = torch.tensor([idx.numel()], dtype=torch.int32, device=DEV)
    out = torch.empty(idx.numel(), F, device=DEV)
    hip.gather_rows(table, idx, n, idx.numel(), out)
    torch.cuda.synchronize()
    assert torch.equal(out, table[ids])
    # fused-gather aggregation: dst d sums rows idx[4d .. 4d+3] with weight 1
    v = idx.numel() // 4
    co = torch.arange(0, 4 * v + 1, 4, dtype=torch.int32, device=DEV)
    ri = torch.arange(4 * v, dtype=torch.int32, device=DEV)
    y = torch.empty(v, F, device=DEV)
    hip.spmm_csc_fwd(co, ri, None, None, v, table, y, row_map=idx)
    r = table[ids].view(v, 4, F)
    ref = ((r[:, 0] + r[:, 1]) + r[:, 2]) + r[:, 3]  # edge order, 1.0 weights
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    W = torch.randn(F, 64, device=DEV, generator=gen)
    C = torch.empty(idx.numel(), 64, device=DEV)
    hip.gemm_gather(table, idx, W, C)
    C2 = torch.empty_like(C)
    hip.gemm(table[ids].contiguous(), W, C2)
    torch.cuda.synchronize()
    assert torch.equal(C, C2)
    del table, out, y, C, C2
    _free()
