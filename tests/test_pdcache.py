"""NeutronOrch PD cache (toolkits/GCN_SAMPLE_PD_CACHE.hpp):
preSample's hot-vertex selection, the omitted bottom-layer sampling, the
shared-embedding load and the driver's super-batch orchestration, against the
oracle's restatements (oracle/ref_cpu.cpp: orc_presample, the sampler's omit
map, orc_pushdown_fwd)."""
import numpy as np
import pytest
import torch

from conftest import GOLDEN
from nts import dataloader
from oracle import oracle as orc

SRC = np.array([0, 2, 1, 3, 4, 1, 0, 4, 3], np.uint32)
DST = np.array([1, 1, 0, 1, 4, 2, 2, 3, 0], np.uint32)


def test_presample_known_answer():
    """get_most_neighbor by hand on the 5-vertex graph (CSC: 0:[1,3] 1:[0,2,3]
    2:[1,0] 3:[4] 4:[4]), seeds {1}."""
    col, rows = orc.build_csc(5, SRC, DST)
    c, ids = orc.presample(col, rows, np.array([1], np.uint32), 2, 0.5)
    # one pass: counts [1,0,1,1,0]; sorted 1,1,1,0,0 -> total 4, n = 2, pivot 1
    assert c.tolist() == [1, 0, 1, 1, 0] and ids.tolist() == [0, 2]
    c, ids = orc.presample(col, rows, np.array([1], np.uint32), 3, 0.5)
    # two passes: [1,2,0,1,1]; sorted 2,1,1,1,0 -> total 5, n = 2, pivot 1
    assert c.tolist() == [1, 2, 0, 1, 1] and ids.tolist() == [0, 1]
    c, ids = orc.presample(col, rows, np.array([1], np.uint32), 3, 0.2)
    # n = 1, pivot = sorted[1] = 1: the first id in id order with count >= 1
    # is 0 — vertex 1 (count 2, above the pivot) is not taken: the reference's
    # selection loop, single thread
    assert ids.tolist() == [0]
    c, ids = orc.presample(col, rows, np.array([1], np.uint32), 1, 0.5)
    assert c.tolist() == [0] * 5 and ids.size == 0  # no pass: all zero, total 1 -> n 0


def test_pushdown_matches_fuse_with_sampled_weights():
    src, dst = dataloader.read_edge_file(GOLDEN / "cora" / "cora.2708.edge.self")
    V = 2708
    col, rows = orc.build_csc(V, src, dst)
    od, idg = orc.degrees(V, src, dst)
    o = orc.Sampler(col, rows, idg, od, [10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    (ly,) = o.sample(np.arange(0, V, 7, dtype=np.uint32))
    X = np.random.default_rng(0).standard_normal((V, 9)).astype(np.float32)
    Y = orc.pushdown_fwd(ly, X, 3, 40)
    # = MiniBatchFuseOp over the gathered rows (Sum weights recomputed identically)
    ref = orc.fuse_fwd(ly, orc.get_feature(ly["source"], X), od, idg)[3:40]
    assert np.array_equal(Y, ref)


def test_oracle_omit_samples_nothing_for_cached_dsts():
    src, dst = dataloader.read_edge_file(GOLDEN / "cora" / "cora.2708.edge.self")
    V = 2708
    col, rows = orc.build_csc(V, src, dst)
    od, idg = orc.degrees(V, src, dst)
    seeds = np.arange(0, V, 31, dtype=np.uint32)
    o = orc.Sampler(col, rows, idg, od, [10, 5], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    full = o.sample(seeds, 4)
    omap = np.full(V, 0xFFFFFFFF, np.uint32)
    hot = full[1]["destination"][::3]
    omap[hot] = 7
    o.set_omit(omap, 7)
    part = o.sample(seeds, 4)
    assert np.array_equal(part[0]["column_offset"], full[0]["column_offset"])  # top layer unchanged
    cnt = np.diff(part[1]["column_offset"].astype(np.int64))
    d = part[1]["destination"]
    assert (cnt[np.isin(d, hot)] == 0).all()
    keep = ~np.isin(d, hot)
    assert np.array_equal(cnt[keep], np.diff(full[1]["column_offset"].astype(np.int64))[keep])


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------
DEV = torch.device("cuda:0")


def _t(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    elif a.dtype == np.uint64:
        a = a.view(np.int64)
    return torch.from_numpy(a).to(DEV)


@pytest.fixture(scope="module")
def hip():
    from nts.hip import HipContext
    return HipContext(0, seed=2000)


def _dev_graph(hip, V, src, dst):
    from nts.hip import DeviceGraph
    s, d = _t(src), _t(dst)
    col, rows = hip.build_csc(s, d, V)
    od, idg = hip.degrees(s, d, V)
    return DeviceGraph(V, src.size, col, rows, idg, od)


@pytest.mark.gpu
@pytest.mark.parametrize("layers,rate", [(2, 0.2), (3, 0.1), (2, 0.9), (1, 0.5), (3, 1.0)])
def test_presample_gpu_matches_oracle(hip, layers, rate):
    src, dst = dataloader.read_edge_file(GOLDEN / "cora" / "cora.2708.edge.self")
    V = 2708
    g = _dev_graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    for seed in range(3):
        seeds = np.random.default_rng(seed).choice(V, 256, replace=False).astype(np.uint32)
        c_ref, ids_ref = orc.presample(col, rows, seeds, layers, rate)
        counts = torch.empty(V, dtype=torch.int32, device=DEV)
        tmp = torch.empty(V, dtype=torch.int32, device=DEV)
        hip.presample_counts(g, _t(seeds), layers, counts, tmp)
        out = torch.empty(V, dtype=torch.int32, device=DEV)
        n = torch.empty(1, dtype=torch.int32, device=DEV)
        hip.presample_select(counts, rate, out, n)
        torch.cuda.synchronize()
        assert np.array_equal(counts.cpu().numpy().view(np.uint32), c_ref)
        assert int(n) == ids_ref.size
        assert np.array_equal(out[:int(n)].cpu().numpy().view(np.uint32), ids_ref)


@pytest.mark.gpu
def test_sampler_omit_matches_oracle_and_records_rows(hip):
    from nts.hip import LayerBuffers, layer_caps
    src, dst = dataloader.read_edge_file(GOLDEN / "cora" / "cora.2708.edge.self")
    V = 2708
    g = _dev_graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    od, idg = orc.degrees(V, src, dst)
    seeds = np.arange(3, V, 29, dtype=np.uint32)
    hot = np.random.default_rng(1).choice(V, 400, replace=False).astype(np.uint32)
    omap = np.full(V, 0xFFFFFFFF, np.uint32)
    oloc = np.zeros(V, np.uint32)
    omap[hot], oloc[hot] = 11, np.arange(hot.size, dtype=np.uint32)
    o = orc.Sampler(col, rows, idg, od, [10, 5], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    o.set_omit(omap, 11)
    ref = o.sample(seeds, 2)
    fan = [10, 5]
    caps = layer_caps(seeds.size, fan, V, src.size)
    hip.reserve(V, max(max(c) for c in caps))
    cur = _t(seeds)
    vsz = torch.tensor([seeds.size], dtype=torch.int32, device=DEV)
    got = []
    om, ol = _t(omap), _t(oloc)
    for l, (f, (vc, ec, sc)) in enumerate(zip(fan, caps)):
        last = l == len(fan) - 1
        lay = LayerBuffers(vc, ec, sc, cur, vsz, DEV, omit_map=om if last else None, omit_key=11,
                           omit_loc=ol if last else None)
        hip.sample_layer(g, lay, f, l, 2, 0, 0)
        got.append(lay)
        cur, vsz = lay.source, lay.sizes[2:3]
    torch.cuda.synchronize()
    for lay, r in zip(got, ref):
        v, e, s, ovf = lay.sizes_host()
        assert ovf == 0 and (v, e, s) == (r["v_size"], r["e_size"], r["src_size"])
        for k in ("column_offset", "row_indices", "sample_ans", "source", "edge_weight_forward"):
            n = {"column_offset": v + 1, "source": s}.get(k, e)
            assert np.array_equal(lay.t[k][:n].cpu().numpy().view(r[k].dtype), r[k]), k
    last = got[-1]
    d = ref[-1]["destination"]
    want = np.where(omap[d] == 11, oloc[d], 0xFFFFFFFF).astype(np.uint32)
    assert np.array_equal(last.t["omit_row"][:d.size].cpu().numpy().view(np.uint32), want)


@pytest.mark.gpu
def test_pd_load_share_and_relu_dropout(hip):
    from test_hip_kernels import _dropout_keep
    rng = np.random.default_rng(5)
    v, F, n = 500, 48, 60
    omit_row = np.full(v, 0xFFFFFFFF, np.uint32)
    pick = rng.choice(v, n, replace=False)
    omit_row[pick] = rng.permutation(n).astype(np.uint32)
    share = rng.standard_normal((n, F)).astype(np.float32)
    Z = rng.standard_normal((v, F)).astype(np.float32)
    z = _t(Z)
    hip.pd_load_share(_t(omit_row), None, v, _t(share), z)
    want = Z.copy()
    want[pick] = share[omit_row[pick]]
    y = torch.empty_like(z)
    p, seed, off = 0.5, 77, 3
    hip.relu_dropout(z, y, p, seed, off)
    torch.cuda.synchronize()
    assert np.array_equal(z.cpu().numpy(), want)
    keep = _dropout_keep(v, F, p, seed, off)
    assert np.array_equal(y.cpu().numpy(), np.where(keep & (want > 0), want * np.float32(2), 0).astype(np.float32))


def _pd_driver(E, graph, rate, **kw):
    from nts import host, synthetic
    feat = synthetic.features(graph["V"], 64, device=DEV)
    labels, masks = synthetic.labels_masks(graph["V"], 7, device=DEV)
    train = torch.nonzero(masks == 0).flatten().to(torch.int32).cpu()
    cfg = host.gcn_config([64, 32, 7], [10, 5], 128, learn_rate=0.01, shuffle=False,
                          transform_first=0, **kw)
    return E.GCN_SAMPLE_ALLGPU_impl(graph["G"], feat, labels, train, cfg), feat, labels, train


@pytest.fixture(scope="module")
def E():
    from nts import host
    return host.ext()


@pytest.fixture(scope="module")
def graph(E):
    from nts import synthetic
    g = synthetic.chung_lu(4000, 120000, 15.0, device=DEV, seed=8)
    G = E.FullyRepGraph.from_edges(g.src, g.dst, g.n_vertices)
    src = g.src.cpu().numpy().view(np.uint32)
    dst = g.dst.cpu().numpy().view(np.uint32)
    col, rows = orc.build_csc(g.n_vertices, src, dst)
    od, idg = orc.degrees(g.n_vertices, src, dst)
    return dict(G=G, V=g.n_vertices, col=col, rows=rows, od=od, idg=idg)


@pytest.mark.gpu
def test_pd_driver_presample_matches_oracle(E, graph):
    drv, *_ , train = _pd_driver(E, graph, 0.3, pd_cache=True, pd_rate=0.3, pd_super_batch=3)
    counts, ids = drv.presample()
    sbs = 128 * 3
    t = train.numpy().astype(np.uint32)
    off = 0
    for b, c in enumerate(counts):
        _, ref = orc.presample(graph["col"], graph["rows"], t[b * sbs:(b + 1) * sbs], 2, 0.3)
        assert np.array_equal(np.array(ids[off:off + c], np.uint32), ref)
        off += c
    assert off == len(ids) and len(counts) == -(-t.size // sbs)


@pytest.mark.gpu
@pytest.mark.parametrize("drop", [0.0, 0.5])
def test_pd_driver_rate_zero_is_plain_training(E, graph, drop):
    """No hot vertices: the PD path (GEMM, empty overwrite, separate
    relu/dropout with the same mask keys) trains to the same weights bit for bit."""
    a, *_ = _pd_driver(E, graph, 0.0, pd_cache=True, pd_rate=0.0, drop_rate=drop)
    b, *_ = _pd_driver(E, graph, 0.0, drop_rate=drop, early_aggregate=False)
    b.set_weights(a.weights())
    for _ in range(4):
        a.train_batch()
        b.train_batch()
    a.synchronize()
    b.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_pd_driver_step_matches_oracle_chain(E, graph):
    """One PD training step (first batch of a super-batch): the oracle samples
    the hot vertices' bottom layer (PushDownBatchOp + X W = the shared
    embedding), the batch with those dsts omitted, and runs the GCN chain with
    their rows of Y W replaced; the loss agrees within fp32 tolerance."""
    drv, feat, labels, train = _pd_driver(E, graph, 0.3, pd_cache=True, pd_rate=0.3,
                                          pd_super_batch=2, drop_rate=0.0)
    counts, ids = drv.presample()
    W0 = [w.cpu() for w in drv.weights()]
    drv.train_batch()
    drv.synchronize()
    loss = float(drv.loss)
    V = graph["V"]
    hot = np.array(ids[:counts[0]], np.uint32)
    X = feat.cpu().numpy()
    # the shared embedding: 1-layer sample of the hot ids (the PD sampler's own stream)
    ps = orc.Sampler(graph["col"], graph["rows"], graph["idg"], graph["od"], [5],
                     rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    (hl,) = ps.sample(hot, 1 << 48)
    share = torch.from_numpy(orc.pushdown_fwd(hl, X)) @ W0[0]
    omap = np.full(V, 0xFFFFFFFF, np.uint32)
    omap[hot] = 1
    o = orc.Sampler(graph["col"], graph["rows"], graph["idg"], graph["od"], [10, 5],
                    rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    o.set_omit(omap, 1)
    l0, l1 = o.sample(train.numpy()[:128].astype(np.uint32), 0)
    Y0 = orc.fuse_fwd(l1, orc.get_feature(l1["source"], X), graph["od"], graph["idg"])
    Z = torch.from_numpy(Y0) @ W0[0]
    pos = {int(v): i for i, v in enumerate(hot)}
    for i, d in enumerate(l1["destination"]):
        if int(d) in pos:
            Z[i] = share[pos[int(d)]]
    X1 = torch.relu(Z)
    Y1 = orc.fuse_fwd(l0, X1.numpy(), graph["od"], graph["idg"])
    out = (torch.from_numpy(Y1) @ W0[1]).log_softmax(1)
    tgt = labels.cpu()[torch.from_numpy(l0["destination"].astype(np.int64))]
    ref = torch.nn.functional.nll_loss(out.log_softmax(1), tgt)
    assert np.isin(l1["destination"], hot).sum() > 10  # the cache is exercised
    assert abs(loss - float(ref)) < 1e-5 * max(1.0, abs(float(ref)))


@pytest.mark.gpu
@pytest.mark.parametrize("cache_rate", [0.0, 0.3])
def test_pd_driver_with_feature_cache_is_identical(E, graph, cache_rate):
    """GS_SAMPLE_PD_CACHE's placement: the feature table in pinned host memory
    with the highest-degree rows cached in HBM.  The PD push-down aggregation
    of the hot vertices then reads the two-tier table too; training is
    bit-identical to the all-HBM table."""
    a, *_ = _pd_driver(E, graph, 0.3, pd_cache=True, pd_rate=0.3, pd_super_batch=2,
                       drop_rate=0.5, early_aggregate=False)
    b, *_ = _pd_driver(E, graph, 0.3, pd_cache=True, pd_rate=0.3, pd_super_batch=2,
                       drop_rate=0.5, early_aggregate=False, cache_rate=cache_rate)
    b.set_weights(a.weights())
    for _ in range(5):
        a.train_batch()
        b.train_batch()
    a.synchronize()
    b.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        assert torch.equal(x, y)
