"""Kernel-level parity of the HIP path (through the C-ABI) against the CPU oracle.

Bar: bit-exact for every integer/index array and for the fp32 aggregation
(same sampCSC, same summation order); atomic scatter within 1e-5 relative.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _t(a, dtype=None):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    elif a.dtype == np.uint64:
        a = a.view(np.int64)
    t = torch.from_numpy(a)
    return t.to(DEV) if dtype is None else t.to(DEV, dtype)


def _np_u32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.fixture(scope="module")
def hip():
    from nts.hip import HipContext
    return HipContext(0, seed=2000)


def _graph(hip, V, src, dst):
    from nts.hip import DeviceGraph
    s, d = _t(src), _t(dst)
    col, rows = hip.build_csc(s, d, V)
    out_d, in_d = hip.degrees(s, d, V)
    torch.cuda.synchronize()
    return DeviceGraph(V, src.size, col, rows, in_d, out_d)


@pytest.fixture(scope="module")
def cora(golden):
    from nts import dataloader
    src, dst = dataloader.read_edge_file(golden / "cora" / "cora.2708.edge.self")
    return 2708, src, dst


def _random_graph(V, E, seed):
    rng = np.random.default_rng(seed)
    # skewed degrees (some hubs), self loops, duplicates allowed
    p = 1.0 / np.arange(1, V + 1) ** 0.8
    p /= p.sum()
    src = rng.choice(V, E, p=p).astype(np.uint32)
    dst = rng.choice(V, E).astype(np.uint32)
    return V, src, dst


@pytest.mark.parametrize("case", ["cora", "random"])
def test_build_csc_and_degrees(hip, cora, case):
    V, src, dst = cora if case == "cora" else _random_graph(5000, 200000, 3)
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    assert np.array_equal(g.column_offset.cpu().numpy().view(np.uint64), col)
    assert np.array_equal(_np_u32(g.row_indices), rows)
    assert np.array_equal(_np_u32(g.out_degree), out_d)
    assert np.array_equal(_np_u32(g.in_degree), in_d)


def _sample_gpu(hip, g, seeds, fanouts, rng_mode, batch_seq=0, weight_type=0, csr=True,
                merge=False):
    from nts.hip import LayerBuffers, layer_caps
    caps = layer_caps(len(seeds), fanouts, g.n_vertices, g.n_edges, merge)
    hip.reserve(g.n_vertices, max(max(c) for c in caps))
    dst = _t(np.asarray(seeds, np.uint32))
    vsz = torch.tensor([len(seeds)], dtype=torch.int32, device=DEV)
    layers = []
    for l, (f, (vc, ec, sc)) in enumerate(zip(fanouts, caps)):
        lay = LayerBuffers(vc, ec, sc, dst, vsz, torch.device(DEV), csr=csr,
                           weights=weight_type != 2, merge=merge)
        hip.sample_layer(g, lay, f, l, batch_seq, rng_mode, weight_type)
        layers.append(lay)
        dst, vsz = lay.source, lay.sizes[2:3]
    torch.cuda.synchronize()
    return layers


def _gpu_layer_np(lay):
    v, e, s, ovf = lay.sizes_host()
    assert ovf == 0
    out = dict(v_size=v, e_size=e, src_size=s,
               destination=_np_u32(lay.destination)[:v],
               column_offset=_np_u32(lay.column_offset)[:v + 1],
               row_indices=_np_u32(lay.row_indices)[:e],
               sample_ans=_np_u32(lay.sample_ans)[:e],
               source=_np_u32(lay.source)[:s])
    if lay.edge_weight_forward is not None:
        out["edge_weight_forward"] = lay.edge_weight_forward.cpu().numpy()[:e]
    if lay.row_offset is not None:
        out["row_offset"] = _np_u32(lay.row_offset)[:s + 1]
        out["column_indices"] = _np_u32(lay.column_indices)[:e]
        if lay.edge_weight_backward is not None:
            out["edge_weight_backward"] = lay.edge_weight_backward.cpu().numpy()[:e]
    if lay.dst_local_id is not None:
        out["dst_local_id"] = _np_u32(lay.dst_local_id)[:v]
    if lay.csr_edge_id is not None:
        out["csr_edge_id"] = _np_u32(lay.csr_edge_id)[:e]
    return out


KEYS = ("destination", "column_offset", "sample_ans", "source", "row_indices", "row_offset",
        "column_indices", "edge_weight_forward", "edge_weight_backward", "dst_local_id",
        "csr_edge_id")


def _assert_layers_equal(gl, ol):
    for a, b in zip(gl, ol):
        assert (a["v_size"], a["e_size"], a["src_size"]) == (b["v_size"], b["e_size"], b["src_size"])
        for k in KEYS:
            if k in a:
                assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("walker", ["serial", "chunked"])
@pytest.mark.parametrize("fanouts", [(25, 10), (3, 2), (-1, 4), (5, 5, 5), (15, 11), (30, 12)])
def test_sampler_mt19937_is_reference_stream(hip, cora, fanouts, walker, monkeypatch):
    """MT19937 mode reproduces the reference generator: identical arrays to the
    oracle in draw order, identical per-dst sets to the reference's
    unordered_map order, identical generator state afterwards — with the
    single-wave walker and with the chunked resolver (bulk words, window
    tables, chained entries, per-chunk replay) forced on every layer."""
    monkeypatch.setenv("NTS_MT_SERIAL" if walker == "serial" else "NTS_MT_CHUNKED", "1")
    V, src, dst = cora
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    rng = np.random.default_rng(1)
    batches = [rng.choice(V, 64, replace=False).astype(np.uint32) for _ in range(3)]
    hip.rng_seed(2000)
    o_draw = orc.Sampler(col, rows, in_d, out_d, list(fanouts), seed=2000,
                         rng_mode=orc.RNG_MT_LEMIRE, order_mode=orc.ORDER_DRAW)
    o_ref = orc.Sampler(col, rows, in_d, out_d, list(fanouts), seed=2000,
                        rng_mode=orc.RNG_MT_LEMIRE, order_mode=orc.ORDER_UNORDERED_MAP)
    for bs, seeds in enumerate(batches):
        gl = [_gpu_layer_np(l) for l in _sample_gpu(hip, g, seeds, list(fanouts), 1, bs)]
        _assert_layers_equal(gl, o_draw.sample(seeds, bs))
        ref = o_ref.sample(seeds, bs)
        for a, b in zip(gl, ref):
            co = a["column_offset"]
            assert np.array_equal(a["source"], b["source"])
            for k in range(a["v_size"]):
                assert sorted(a["sample_ans"][co[k]:co[k + 1]]) == sorted(b["sample_ans"][co[k]:co[k + 1]])
    assert np.array_equal(hip.rng_state().numpy().view(np.uint32), o_draw.mt_state())


def _regular_graph(V, d, seed):
    """Every vertex with exactly d distinct in-neighbours."""
    rng = np.random.default_rng(seed)
    src = np.concatenate([rng.choice(V, d, replace=False) for _ in range(V)]).astype(np.uint32)
    dst = np.repeat(np.arange(V, dtype=np.uint32), d)
    return V, src, dst


@pytest.mark.parametrize("walker", ["serial", "chunked"])
@pytest.mark.parametrize("deg,fanouts", [(26, (25, 25)), (11, (10, 10))])
def test_sampler_mt19937_coupon_collector(hip, deg, fanouts, walker, monkeypatch):
    """Every degree = fanout + 1, the worst case of the rejection draws (about
    3x the words of the sampled edges at fanout 25: the coupon collector):
    the stream generated for each layer covers it — arrays bit-exact vs the
    oracle's std::mt19937(2000) walk and the generator state identical after
    every batch (core/ntsFastSampler.hpp:200-205,1020-1054)."""
    monkeypatch.setenv("NTS_MT_SERIAL" if walker == "serial" else "NTS_MT_CHUNKED", "1")
    V, src, dst = _regular_graph(30_000, deg, 4)
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    rng = np.random.default_rng(2)
    hip.rng_seed(2000)
    o = orc.Sampler(col, rows, in_d, out_d, list(fanouts), seed=2000,
                    rng_mode=orc.RNG_MT_LEMIRE, order_mode=orc.ORDER_DRAW)
    for bs in range(2):
        seeds = rng.choice(V, 2048, replace=False).astype(np.uint32)
        gl = [_gpu_layer_np(l) for l in _sample_gpu(hip, g, seeds, list(fanouts), 1, bs)]
        _assert_layers_equal(gl, o.sample(seeds, bs))
        assert np.array_equal(hip.rng_state().numpy().view(np.uint32), o.mt_state()), bs


def test_sampler_mt19937_div_mode(hip, cora):
    V, src, dst = cora
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    seeds = np.arange(5, 2708, 41, dtype=np.uint32)
    hip.rng_seed(2000)
    o = orc.Sampler(col, rows, in_d, out_d, [10, 5], seed=2000, rng_mode=orc.RNG_MT_DIV,
                    order_mode=orc.ORDER_DRAW)
    gl = [_gpu_layer_np(l) for l in _sample_gpu(hip, g, seeds, [10, 5], 2)]
    _assert_layers_equal(gl, o.sample(seeds))


def _hub_graph(seed):
    """Degrees past the 1024 rejection-set cap and past the MT exact path's
    16 K direct table: 48 hub dsts of 20,000 in-edges, 400 of 1,500-3,000,
    and a sparse rest."""
    rng = np.random.default_rng(seed)
    V = 60_000
    parts_s, parts_d = [], []
    for d in range(48):
        parts_s.append(rng.integers(0, V, 20_000))
        parts_d.append(np.full(20_000, d))
    for d in range(48, 448):
        k = int(rng.integers(1_500, 3_000))
        parts_s.append(rng.integers(0, V, k))
        parts_d.append(np.full(k, d))
    parts_s.append(rng.integers(0, V, 300_000))
    parts_d.append(rng.integers(0, V, 300_000))
    return V, np.concatenate(parts_s).astype(np.uint32), np.concatenate(parts_d).astype(np.uint32)


@pytest.mark.parametrize("rng_mode", [0, 1])
def test_sampler_fanout_above_1024(hip, rng_mode):
    """Fanout 2,000 (> the 1,024-entry rejection set): the LDS hash-set path
    (Philox) and the MT exact paths (direct table, hashed past 16 K degree)
    give the oracle's arrays in draw order (std::unordered_map semantics,
    core/ntsFastSampler.hpp:1028-1048), and the MT generator state matches."""
    V, src, dst = _hub_graph(12)
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    seeds = np.concatenate([np.arange(0, 448, 3), np.arange(1000, 1200)]).astype(np.uint32)
    fan = [2000, 3]
    hip.rng_seed(2000)
    o = orc.Sampler(col, rows, in_d, out_d, fan, seed=2000,
                    rng_mode=orc.RNG_PHILOX if rng_mode == 0 else orc.RNG_MT_LEMIRE,
                    order_mode=orc.ORDER_DRAW)
    for bs in range(2):
        gl = [_gpu_layer_np(l) for l in _sample_gpu(hip, g, seeds, fan, rng_mode, bs)]
        ol = o.sample(seeds, bs)
        assert ol[0]["e_size"] > 100 * 2000
        _assert_layers_equal(gl, ol)
    if rng_mode == 1:
        assert np.array_equal(hip.rng_state().numpy().view(np.uint32), o.mt_state())


@pytest.mark.parametrize("case", ["cora", "random"])
@pytest.mark.parametrize("weight_type", [0, 1, 2, 3, 0x10, 0x11, 0x13])  # 0x10: UP_DEGREE, 3: MEAN_SAMPLED
def test_sampler_philox_matches_oracle(hip, cora, case, weight_type):
    V, src, dst = cora if case == "cora" else _random_graph(20000, 600000, 9)
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    rng = np.random.default_rng(2)
    seeds = rng.choice(V, min(V, 512), replace=False).astype(np.uint32)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], seed=2000, rng_mode=orc.RNG_PHILOX,
                    order_mode=orc.ORDER_DRAW)
    for bs in (0, 7):
        gl = [_gpu_layer_np(l) for l in _sample_gpu(hip, g, seeds, [25, 10], 0, bs, weight_type)]
        ol = o.sample(seeds, bs, weight_type)
        if weight_type == 2:
            for x in ol:
                x.pop("edge_weight_forward"), x.pop("edge_weight_backward")
        _assert_layers_equal(gl, ol)


@pytest.mark.parametrize("case", ["cora", "random"])
def test_sampler_merge_src_dst_matches_oracle(hip, cora, case):
    """is_merge_src_dst (GAT drivers): dsts join the frontier, dst_local_id maps
    each dst to its local src id, CSR slots carry their CSC edge ids."""
    V, src, dst = cora if case == "cora" else _random_graph(20000, 600000, 9)
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    seeds = np.random.default_rng(4).choice(V, min(V, 512), replace=False).astype(np.uint32)
    o = orc.Sampler(col, rows, in_d, out_d, [10, 5], seed=2000, rng_mode=orc.RNG_PHILOX,
                    order_mode=orc.ORDER_DRAW)
    gl = [_gpu_layer_np(l) for l in _sample_gpu(hip, g, seeds, [10, 5], 0, 3, 0, merge=True)]
    ol = o.sample(seeds, 3, orc.W_SUM | orc.F_MERGE_SRC_DST)
    for a, b in zip(gl, ol):
        assert "dst_local_id" in a and "csr_edge_id" in a and "dst_local_id" in b
        assert np.array_equal(a["source"][a["dst_local_id"]], a["destination"])
    _assert_layers_equal(gl, ol)


def test_sampler_edge_cases(hip):
    # empty batch, isolated vertices (self loop only), fanout 0, hub above 1024
    V = 3000
    src = np.concatenate([np.arange(V), np.zeros(2000), np.arange(1, 2001)]).astype(np.uint32)
    dst = np.concatenate([np.arange(V), np.arange(1, 2001), np.zeros(2000)]).astype(np.uint32)
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    for seeds, fan in [(np.array([], np.uint32), [4, 4]), (np.array([0, 2999, 5], np.uint32), [0, 3]),
                       (np.array([0], np.uint32), [1500, 2]), (np.array([0, 7], np.uint32), [-1, -1]),
                       (np.array([0], np.uint32), [20000, 2])]:
        o = orc.Sampler(col, rows, in_d, out_d, fan, rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
        if any(f > 16384 for f in fan):  # past the distinct-position hash set
            with pytest.raises(RuntimeError):
                _sample_gpu(hip, g, seeds, fan, 0)
            continue
        gl = [_gpu_layer_np(l) for l in _sample_gpu(hip, g, seeds, fan, 0)]
        _assert_layers_equal(gl, o.sample(seeds))


@pytest.mark.parametrize("F", [1, 7, 41, 100, 128, 256, 602, 1433])
def test_spmm_fwd_bitexact_and_fused_gather(hip, cora, F):
    V, src, dst = cora
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    seeds = np.arange(0, V, 11, dtype=np.uint32)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, l1 = o.sample(seeds)
    rng = np.random.default_rng(F)
    table = rng.standard_normal((V, F)).astype(np.float32)
    X = orc.get_feature(l1["source"], table)
    Y_ref = orc.fuse_fwd(l1, X, out_d, in_d)
    v = l1["v_size"]
    co, ri, wf = _t(l1["column_offset"]), _t(l1["row_indices"]), _t(l1["edge_weight_forward"])
    vdev = torch.tensor([v], dtype=torch.int32, device=DEV)
    y = torch.full((v + 5, F), float("nan"), device=DEV)
    hip.spmm_csc_fwd(co, ri, wf, vdev, v + 5, _t(X), y)
    torch.cuda.synchronize()
    assert np.array_equal(y[:v].cpu().numpy(), Y_ref)
    assert torch.isnan(y[v:]).all()  # rows past the live size untouched
    # fused gather: rows straight from the feature table through `source`
    y2 = torch.empty((v, F), device=DEV)
    hip.spmm_csc_fwd(co, ri, wf, vdev, v, _t(table), y2, row_map=_t(l1["source"]))
    # gather_rows == get_feature
    x0 = torch.empty((l1["src_size"], F), device=DEV)
    n = torch.tensor([l1["src_size"]], dtype=torch.int32, device=DEV)
    hip.gather_rows(_t(table), _t(l1["source"]), n, l1["src_size"], x0)
    torch.cuda.synchronize()
    assert np.array_equal(y2.cpu().numpy(), Y_ref)
    assert np.array_equal(x0.cpu().numpy(), X)
    # padded pitches (the 128-byte feature / output layout): float4 loads with a
    # partial last vector; the pitch padding of the output stays untouched
    if F % 4:
        pad = (F + 31) // 32 * 32
        tp = torch.full((V, pad), float("nan"), device=DEV)
        tp[:, :F] = _t(table)
        y3 = torch.full((v, pad), 7.0, device=DEV)
        hip.spmm_csc_fwd(co, ri, wf, vdev, v, tp[:, :F], y3[:, :F], row_map=_t(l1["source"]))
        torch.cuda.synchronize()
        assert np.array_equal(y3[:, :F].cpu().numpy(), Y_ref)
        assert (y3[:, F:] == 7.0).all()


def _assert_csr_rows(got, ref, row_offset):
    """CSR gathers: rows of at most 16 edges keep the serial edge order of
    MiniBatchFuseOp::backward (bit-exact); longer rows are summed as in-order
    pieces by the whole workgroup (deterministic, fp32 summation order)."""
    ln = np.diff(row_offset.astype(np.int64))
    short = ln <= 16
    assert short.any()
    assert np.array_equal(got[short], ref[short])
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("F", [16, 41, 128, 256, 602])
def test_spmm_backward_csr_bitexact_and_atomic(hip, cora, F):
    V, src, dst = cora
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, _ = o.sample(np.arange(3, V, 17, dtype=np.uint32))
    rng = np.random.default_rng(F)
    G = rng.standard_normal((l0["v_size"], F)).astype(np.float32)
    Gin_ref = orc.fuse_bwd(l0, G, out_d, in_d)
    s = l0["src_size"]
    sdev = torch.tensor([s], dtype=torch.int32, device=DEV)
    gin = torch.empty((s, F), device=DEV)
    hip.spmm_csr_bwd(_t(l0["row_offset"]), _t(l0["column_indices"]), _t(l0["edge_weight_backward"]),
                     sdev, s, _t(G), gin)
    vdev = torch.tensor([l0["v_size"]], dtype=torch.int32, device=DEV)
    gat = torch.zeros((s, F), device=DEV)
    hip.spmm_csc_bwd_atomic(_t(l0["column_offset"]), _t(l0["row_indices"]),
                            _t(l0["edge_weight_forward"]), vdev, l0["v_size"], _t(G), gat)
    torch.cuda.synchronize()
    _assert_csr_rows(gin.cpu().numpy(), Gin_ref, l0["row_offset"])
    np.testing.assert_allclose(gat.cpu().numpy(), Gin_ref, rtol=1e-5, atol=1e-6)


def test_gather_labels(hip):
    lab = torch.arange(1000, dtype=torch.int64, device=DEV) * 3
    idx = torch.randint(0, 1000, (777,), dtype=torch.int32, device=DEV)
    out = torch.empty(777, dtype=torch.int64, device=DEV)
    n = torch.tensor([777], dtype=torch.int32, device=DEV)
    hip.gather_labels(lab, idx, n, 777, out)
    torch.cuda.synchronize()
    assert torch.equal(out, lab[idx.long()])


@pytest.mark.parametrize("bias_correction", [True, False])
def test_adam_matches_reference_torch_expressions(hip, bias_correction):
    rng = np.random.default_rng(4)
    W0 = rng.standard_normal((602, 128)).astype(np.float32)
    G0 = rng.standard_normal((602, 128)).astype(np.float32) * 1e-2
    alpha, b1, b2, eps, wd = np.float32(0.001), np.float32(0.9), np.float32(0.999), np.float32(1e-9), np.float32(1e-4)
    W, M, Vv = torch.from_numpy(W0.copy()), torch.zeros(602, 128), torch.zeros(602, 128)
    w, m, v = _t(W0), torch.zeros(602, 128, device=DEV), torch.zeros(602, 128, device=DEV)
    b1t, b2t = np.float32(b1), np.float32(b2)
    for step in range(3):
        G = torch.from_numpy(G0 * (step + 1))
        if bias_correction:  # Parameter::learnC2C_with_decay_Adam (core/NtsScheduler.hpp:863-880)
            Wg = G + float(wd) * W
            M = float(b1) * M + float(np.float32(1) - b1) * Wg
            Vv = float(b2) * Vv + float(np.float32(1) - b2) * torch.square(Wg)
            Mt = M / float(np.float32(1) - b1t)
            Vt = Vv / float(np.float32(1) - b2t)
            W = W - float(alpha) * Mt / (torch.sqrt(Vt) + float(eps))
        else:  # Parameter::learn_local_with_decay_Adam (core/NtsScheduler.hpp:937-945)
            Wg = W * float(wd)
            Wg = Wg + G
            M = float(b1) * M + float(np.float32(1) - b1) * Wg
            Vv = float(b2) * Vv + float(np.float32(1) - b2) * Wg * Wg
            W = W - float(alpha) * M / (torch.sqrt(Vv) + float(eps))
        hip.adam(w, _t(G.numpy()), m, v, float(alpha), float(b1), float(b2), float(eps), float(wd),
                 float(b1t), float(b2t), bias_correction)
        b1t, b2t = np.float32(b1t * b1), np.float32(b2t * b2)
    torch.cuda.synchronize()
    # torch's CPU sqrt is not correctly rounded on AVX512 hosts (1-ulp
    # differences that then feed the next step), so the kernel is compared
    # bit-exactly with an IEEE float32 restatement of the same expressions and
    # to fp32 tolerance with the reference's torch expressions.
    torch.testing.assert_close(w.cpu(), W, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(m.cpu(), M, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(v.cpu(), Vv, rtol=1e-5, atol=1e-12)
    Wn, Mn, Vn = W0.copy(), np.zeros_like(W0), np.zeros_like(W0)
    b1t, b2t = np.float32(b1), np.float32(b2)
    one = np.float32(1)
    for step in range(3):
        Gn = G0 * np.float32(step + 1)
        if bias_correction:
            wg = Gn + wd * Wn
            Mn = b1 * Mn + (one - b1) * wg
            Vn = b2 * Vn + (one - b2) * (wg * wg)
            Wn = Wn - (alpha * (Mn / (one - b1t))) / (np.sqrt(Vn / (one - b2t)) + eps)
        else:
            wg = Wn * wd + Gn
            Mn = b1 * Mn + (one - b1) * wg
            Vn = b2 * Vn + ((one - b2) * wg) * wg
            Wn = Wn - (alpha * Mn) / (np.sqrt(Vn) + eps)
        b1t, b2t = np.float32(b1t * b1), np.float32(b2t * b2)
    assert np.array_equal(w.cpu().numpy(), Wn)
    assert np.array_equal(m.cpu().numpy(), Mn)
    assert np.array_equal(v.cpu().numpy(), Vn)


@pytest.mark.parametrize("M,N,K", [(150000, 128, 602), (1000, 41, 128), (333, 7, 1433),
                                   (5, 256, 100), (10000, 47, 256), (1, 1, 1), (64, 128, 0),
                                   # LDS-resident-weight NN / row-streaming TN kernels:
                                   # odd K, 128-column slices, narrow N, tails
                                   (4097, 128, 301), (3001, 256, 200), (2100, 64, 602),
                                   (333, 256, 5000), (700, 128, 3)])
@pytest.mark.parametrize("trans_a", [False, True])
def test_gemm_f32_mfma(hip, M, N, K, trans_a):
    """MFMA fp32 GEMM vs torch fp64 (asymmetric data, ragged tails, long split
    reductions).  Products are exact fp32, sums fp32 in a fixed order."""
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + K)
    if trans_a:  # C[M,N] = A[K,M]^T B[K,N]
        A = torch.randn(K, M, device=DEV, generator=g)
    else:
        A = torch.randn(M, K, device=DEV, generator=g)
    B = torch.randn(K, N, device=DEV, generator=g) + torch.arange(N, device=DEV) * 0.01
    C = torch.full((M, N), float("nan"), device=DEV)
    hip.gemm(A, B, C, trans_a=trans_a)
    ref = (A.double().t() if trans_a else A.double()) @ B.double()
    torch.cuda.synchronize()
    tol = 2e-6 * max(K, 1) ** 0.5 + 1e-6
    torch.testing.assert_close(C.double(), ref, rtol=tol, atol=tol * 4)
    # deterministic: a second run is bit-identical
    C2 = torch.empty_like(C)
    hip.gemm(A, B, C2, trans_a=trans_a)
    torch.cuda.synchronize()
    assert torch.equal(C, C2)


@pytest.mark.parametrize("F", [1, 7, 41, 128, 256, 602])
@pytest.mark.parametrize("p", [0.0, 0.5])
def test_spmm_fwd_act_bitexact(hip, cora, F, p):
    """Transform-first aggregation with vertexForward's activation in the
    epilogue: dropout(relu(A x)) == the oracle's MiniBatchFuseOp sum followed by
    the documented Philox keep mask (the GEMM epilogue's keys), bit for bit."""
    V, src, dst = cora
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, l1 = o.sample(np.arange(1, V, 9, dtype=np.uint32))
    rng = np.random.default_rng(F + 100)
    X = rng.standard_normal((l1["src_size"], F)).astype(np.float32)
    Y = orc.fuse_fwd(l1, X, out_d, in_d)
    v = l1["v_size"]
    seed, offset = 0x0123_4567_89AB, 9
    keep = _dropout_keep(v, F, p, seed, offset)
    scale = np.float32(1.0 / (1.0 - p))
    ref = np.where(keep & (Y > 0), Y * scale, np.float32(0)).astype(np.float32)
    vdev = torch.tensor([v], dtype=torch.int32, device=DEV)
    y = torch.full((v + 3, F), float("nan"), device=DEV)
    hip.spmm_csc_fwd_act(_t(l1["column_offset"]), _t(l1["row_indices"]),
                         _t(l1["edge_weight_forward"]), vdev, v + 3, _t(X), y, p=p, seed=seed,
                         offset=offset)
    torch.cuda.synchronize()
    assert np.array_equal(y[:v].cpu().numpy(), ref)
    assert torch.isnan(y[v:]).all()


@pytest.mark.parametrize("F", [1, 7, 41, 128, 602])
def test_spmm_csr_bwd_masked(hip, cora, F):
    """Its backward: A^T (G ⊙ [X > 0] * scale) over the CSR == the oracle's
    dst-ordered MiniBatchFuseOp::backward of the masked gradient."""
    V, src, dst = cora
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    _, l1 = o.sample(np.arange(2, V, 13, dtype=np.uint32))
    rng = np.random.default_rng(F + 7)
    v, s = l1["v_size"], l1["src_size"]
    G = rng.standard_normal((v, F)).astype(np.float32)
    Xa = np.maximum(rng.standard_normal((v, F)).astype(np.float32), 0) * np.float32(2)
    dZ = np.where(Xa > 0, G * np.float32(2.0), np.float32(0)).astype(np.float32)
    ref = orc.fuse_bwd(l1, dZ, out_d, in_d)
    sdev = torch.tensor([s], dtype=torch.int32, device=DEV)
    gin = torch.full((s + 2, F), float("nan"), device=DEV)
    hip.spmm_csr_bwd_masked(_t(l1["row_offset"]), _t(l1["column_indices"]),
                            _t(l1["edge_weight_backward"]), sdev, s + 2, _t(G), _t(Xa), gin,
                            scale=2.0)
    torch.cuda.synchronize()
    _assert_csr_rows(gin[:s].cpu().numpy(), ref, l1["row_offset"])
    assert torch.isnan(gin[s:]).all()


@pytest.mark.parametrize("F", [1, 41, 128, 256, 602])
def test_spmm_csr_bwd_postmask(hip, cora, F):
    """The graph-op backward with the next layer's activation backward fused on
    its output rows == the CSR backward followed by act_backward, bit for bit."""
    V, src, dst = cora
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, _ = o.sample(np.arange(4, V, 11, dtype=np.uint32))
    rng = np.random.default_rng(F + 3)
    v, s = l0["v_size"], l0["src_size"]
    G = _t(rng.standard_normal((v, F)).astype(np.float32))
    Xa = _t((np.maximum(rng.standard_normal((s, F)), 0) * 2).astype(np.float32))
    sdev = torch.tensor([s], dtype=torch.int32, device=DEV)
    ro, ci, wb = _t(l0["row_offset"]), _t(l0["column_indices"]), _t(l0["edge_weight_backward"])
    plain = torch.empty(s, F, device=DEV)
    hip.spmm_csr_bwd(ro, ci, wb, sdev, s, G, plain)
    ref = torch.empty(s, F, device=DEV)
    hip.act_backward(plain, Xa, ref, scale=2.0)
    got = torch.full((s + 2, F), float("nan"), device=DEV)
    hip.spmm_csr_bwd_postmask(ro, ci, wb, sdev, s + 2, G, Xa, got, scale=2.0)
    torch.cuda.synchronize()
    assert torch.equal(got[:s], ref)
    assert torch.isnan(got[s:]).all()


@pytest.mark.gpu
def test_spmm_csr_bwd_postmask_many_rows(hip):
    """The post-mask CSR gather at hop-0 scale (200,000 rows of ~2 edges, empty
    rows, and hub rows of 33-3,000 edges scattered over the blocks): a lane
    group may take several rows (capped grid) — bit-identical to the plain CSR
    backward (one row per group) followed by act_backward."""
    g = torch.Generator(device=DEV).manual_seed(11)
    s, v, F = 200_000, 10_000, 128
    ln = torch.poisson(torch.full((s,), 1.8, device=DEV), generator=g).to(torch.int64)
    hubs = torch.randint(0, s, (300,), device=DEV, generator=g)
    ln[hubs] = torch.randint(33, 3000, (300,), device=DEV, generator=g)
    ln[hubs[:40] // 64 * 64] = 40  # several long rows in one block
    ro = torch.zeros(s + 1, dtype=torch.int64, device=DEV)
    ro[1:] = torch.cumsum(ln, 0)
    e = int(ro[-1])
    ci = torch.randint(0, v, (e,), device=DEV, generator=g).to(torch.int32)
    wb = torch.rand(e, device=DEV, generator=g)
    ro = ro.to(torch.int32)
    G = torch.randn(v, F, device=DEV, generator=g)
    Xa = torch.relu(torch.randn(s, F, device=DEV, generator=g)) * 2
    sdev = torch.tensor([s], dtype=torch.int32, device=DEV)
    plain = torch.empty(s, F, device=DEV)
    hip.spmm_csr_bwd(ro, ci, wb, sdev, s, G, plain)
    ref = torch.empty(s, F, device=DEV)
    hip.act_backward(plain, Xa, ref, scale=2.0)
    got = torch.full((s + 5, F), float("nan"), device=DEV)
    hip.spmm_csr_bwd_postmask(ro, ci, wb, sdev, s + 5, G, Xa, got, scale=2.0)
    torch.cuda.synchronize()
    assert torch.equal(got[:s], ref)
    assert torch.isnan(got[s:]).all()


def _pack_act_bits(y, words):
    """The keep mask [y > 0] in nts_hip_act_bits_words' layout: column j is
    float4 f = j // 4, component q = j % 4, on lane l = f % LPD of chunk
    c = f // LPD (LPD 32 up to 32 float4, else 64), word (h NCH + c) 4 + q with
    h = l // 32, bit l % 32."""
    rows, F = y.shape
    nv = F // 4
    lpd = 32 if nv <= 32 else 64
    nch = 1 if lpd == 32 else (nv + 63) // 64
    assert words == (lpd // 32) * nch * 4
    j = np.arange(F)
    f4, q = j // 4, j % 4
    c, l = f4 // lpd, f4 % lpd
    word = ((l // 32) * nch + c) * 4 + q
    out = np.zeros((rows, words), dtype=np.uint64)
    keep = (y > 0).astype(np.uint64)
    for k in range(F):
        out[:, word[k]] |= keep[:, k] << np.uint64(l[k] % 32)
    return out.astype(np.uint32)


def test_act_bits_words(hip):
    assert [hip.act_bits_words(F) for F in (68, 128, 132, 256, 512, 1024, 2048)] == [4, 4, 8, 8, 16, 32, 64]
    assert [hip.act_bits_words(F) for F in (0, 4, 41, 64, 130, 602, 2052)] == [0] * 7


@pytest.mark.parametrize("F", [68, 128, 256, 512])
def test_spmm_csc_fwd_act_bits(hip, cora, F):
    """The forward that also writes its keep mask as bits: the output equal to
    spmm_csc_fwd_act's, the bits equal to [y > 0] in the documented layout."""
    V, src, dst = cora
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    _, l1 = o.sample(np.arange(2, V, 13, dtype=np.uint32))
    rng = np.random.default_rng(F)
    v, s = l1["v_size"], l1["src_size"]
    X = _t(rng.standard_normal((s, F)).astype(np.float32))
    vdev = torch.tensor([v], dtype=torch.int32, device=DEV)
    args = (_t(l1["column_offset"]), _t(l1["row_indices"]), _t(l1["edge_weight_forward"]), vdev, v + 3, X)
    ref = torch.empty(v + 3, F, device=DEV)
    hip.spmm_csc_fwd_act(*args, ref, p=0.5, seed=9, offset=2)
    W = hip.act_bits_words(F)
    y = torch.empty(v + 3, F, device=DEV)
    bits = torch.full(((v + 3) * W,), -1, dtype=torch.int32, device=DEV)
    hip.spmm_csc_fwd_act_bits(*args, y, bits, p=0.5, seed=9, offset=2)
    torch.cuda.synchronize()
    assert torch.equal(y[:v], ref[:v])
    got = bits.view(v + 3, W)[:v].cpu().numpy().view(np.uint32)
    assert np.array_equal(got, _pack_act_bits(y[:v].cpu().numpy(), W))
    assert (bits.view(v + 3, W)[v:] == -1).all()  # rows past v untouched


@pytest.mark.parametrize("F", [68, 128, 256, 512])
def test_spmm_csr_bwd_postmask_bits(hip, cora, F):
    """The post-mask CSR backward reading the forward's mask bits == the same
    backward reading the forward's output rows, bit for bit."""
    V, src, dst = cora
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, l1 = o.sample(np.arange(4, V, 11, dtype=np.uint32))
    rng = np.random.default_rng(F + 5)
    # the bottom layer l1 (dsts = l0's srcs) makes the activation, l0 backward reads it
    v1, s1 = l1["v_size"], l1["src_size"]
    X = _t(rng.standard_normal((s1, F)).astype(np.float32))
    W = hip.act_bits_words(F)
    Xa = torch.empty(v1, F, device=DEV)
    bits = torch.empty(v1 * W, dtype=torch.int32, device=DEV)
    hip.spmm_csc_fwd_act_bits(_t(l1["column_offset"]), _t(l1["row_indices"]), _t(l1["edge_weight_forward"]),
                              torch.tensor([v1], dtype=torch.int32, device=DEV), v1, X, Xa, bits,
                              p=0.3, seed=4, offset=1)
    v, s = l0["v_size"], l0["src_size"]
    assert s == v1
    G = _t(rng.standard_normal((v, F)).astype(np.float32))
    sdev = torch.tensor([s], dtype=torch.int32, device=DEV)
    ro, ci, wb = _t(l0["row_offset"]), _t(l0["column_indices"]), _t(l0["edge_weight_backward"])
    ref = torch.empty(s, F, device=DEV)
    hip.spmm_csr_bwd_postmask(ro, ci, wb, sdev, s, G, Xa, ref, scale=1.0 / 0.7)
    got = torch.full((s + 2, F), float("nan"), device=DEV)
    hip.spmm_csr_bwd_postmask_bits(ro, ci, wb, sdev, s + 2, G, bits, got, scale=1.0 / 0.7)
    torch.cuda.synchronize()
    assert torch.equal(got[:s], ref)
    assert torch.isnan(got[s:]).all()


@pytest.mark.gpu
def test_spmm_csr_bwd_postmask_bits_many_rows(hip):
    """The bits form at hop-0 scale with hub rows (block-cooperative sums)."""
    g = torch.Generator(device=DEV).manual_seed(12)
    s, v, F = 200_000, 10_000, 128
    ln = torch.poisson(torch.full((s,), 1.8, device=DEV), generator=g).to(torch.int64)
    hubs = torch.randint(0, s, (300,), device=DEV, generator=g)
    ln[hubs] = torch.randint(33, 3000, (300,), device=DEV, generator=g)
    ro = torch.zeros(s + 1, dtype=torch.int64, device=DEV)
    ro[1:] = torch.cumsum(ln, 0)
    e = int(ro[-1])
    ci = torch.randint(0, v, (e,), device=DEV, generator=g).to(torch.int32)
    wb = torch.rand(e, device=DEV, generator=g)
    ro = ro.to(torch.int32)
    G = torch.randn(v, F, device=DEV, generator=g)
    Xa = torch.relu(torch.randn(s, F, device=DEV, generator=g))
    W = hip.act_bits_words(F)
    bits = torch.from_numpy(_pack_act_bits(Xa.cpu().numpy(), W).view(np.int32)).to(DEV).reshape(-1)
    sdev = torch.tensor([s], dtype=torch.int32, device=DEV)
    ref = torch.empty(s, F, device=DEV)
    hip.spmm_csr_bwd_postmask(ro, ci, wb, sdev, s, G, Xa, ref, scale=2.0)
    got = torch.empty(s, F, device=DEV)
    hip.spmm_csr_bwd_postmask_bits(ro, ci, wb, sdev, s, G, bits, got, scale=2.0)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("F", [4, 40, 128, 512])
def test_spmm_csr_bwd_colmax(hip, cora, F):
    """The CSR backward that also emits its output's column maxima per part of
    R rows for the pair-table TN GEMM: the rows bit-identical to
    spmm_csr_bwd's, every part's maxima exact (hub rows summed cooperatively
    included), parts past the live rows zero."""
    V, src, dst = cora
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, _ = o.sample(np.arange(4, V, 11, dtype=np.uint32))
    rng = np.random.default_rng(F + 5)
    v, s = l0["v_size"], l0["src_size"]
    G = _t(rng.standard_normal((v, F)).astype(np.float32))
    sdev = torch.tensor([s], dtype=torch.int32, device=DEV)
    ro, ci, wb = _t(l0["row_offset"]), _t(l0["column_indices"]), _t(l0["edge_weight_backward"])
    plain = torch.empty(s, F, device=DEV)
    hip.spmm_csr_bwd(ro, ci, wb, sdev, s, G, plain)
    cap = s + 37
    R = hip.colmax_rows_per_part(F)
    nparts = (cap + R - 1) // R
    got = torch.full((cap, F), float("nan"), device=DEV)
    parts = torch.full((nparts, F), -1, dtype=torch.int32, device=DEV)
    hip.spmm_csr_bwd_colmax(ro, ci, wb, sdev, cap, G, got, parts)
    torch.cuda.synchronize()
    assert torch.equal(got[:s], plain)
    pad = torch.zeros(nparts * R, F, device=DEV)
    pad[:s] = plain.abs()
    want = pad.view(nparts, R, F).max(1).values
    assert torch.equal(parts.view(torch.float32), want)
    # scaled by power-of-two row scales through a row map (the pair table's
    # rs[source[s]], the TN GEMM's exact operand maxima)
    rsv = torch.pow(2.0, torch.randint(-30, 30, (V,), device=DEV).float())
    rmap = _t(l0["source"])
    parts2 = torch.full((nparts, F), -1, dtype=torch.int32, device=DEV)
    got2 = torch.empty_like(got)
    hip.spmm_csr_bwd_colmax(ro, ci, wb, sdev, cap, G, got2, parts2, rs=rsv, rows=rmap)
    torch.cuda.synchronize()
    assert torch.equal(got2[:s], plain)
    pad[:s] = plain.abs() * rsv[rmap.long()][:, None]
    assert torch.equal(parts2.view(torch.float32), pad.view(nparts, R, F).max(1).values)


@pytest.mark.parametrize("M,N,K", [(3000, 128, 602), (2500, 64, 100), (500, 41, 100), (37, 7, 13)])
def test_gemm_gather_rows(hip, M, N, K):
    """C = table[rows] @ W with the rows gathered inside the GEMM: bit-identical
    to the GEMM on the gathered copy, fp32-accurate vs fp64."""
    g = torch.Generator(device=DEV).manual_seed(M + K)
    V = 4 * M + 11
    ld = (K + 31) // 32 * 32 if K >= 256 else K
    table = torch.randn(V, ld, device=DEV, generator=g)[:, :K]
    rows = torch.randperm(V, device=DEV, generator=g)[:M].to(torch.int32)
    W = torch.randn(K, N, device=DEV, generator=g)
    C = torch.empty(M, N, device=DEV)
    hip.gemm_gather(table, rows, W, C)
    Xg = table[rows.long()].contiguous()
    C2 = torch.empty(M, N, device=DEV)
    hip.gemm(Xg, W, C2)
    torch.cuda.synchronize()
    assert torch.equal(C, C2)
    tol = 2e-6 * K ** 0.5 + 1e-6
    torch.testing.assert_close(C.double(), Xg.double() @ W.double(), rtol=tol, atol=tol * 4)


@pytest.mark.parametrize("M,N,K", [(602, 128, 5000), (100, 256, 3000), (41, 7, 300), (602, 128, 17)])
def test_gemm_tn_gather_rows(hip, M, N, K):
    """dW = table[rows]^T @ G (the transform-first weight gradient): bit-identical
    to the TN GEMM on the gathered copy, fp32-accurate vs fp64."""
    g = torch.Generator(device=DEV).manual_seed(M * N + K)
    V = 3 * K + 5
    ld = (M + 31) // 32 * 32 if M >= 256 else M
    table = torch.randn(V, ld, device=DEV, generator=g)[:, :M]
    rows = torch.randint(0, V, (K,), device=DEV, generator=g).to(torch.int32)
    G = torch.randn(K, N, device=DEV, generator=g)
    C = torch.empty(M, N, device=DEV)
    hip.gemm_tn_gather(table, rows, G, C)
    Xg = table[rows.long()].contiguous()
    C2 = torch.empty(M, N, device=DEV)
    hip.gemm(Xg, G, C2, trans_a=True)
    torch.cuda.synchronize()
    tol = 2e-6 * K ** 0.5 + 1e-6
    torch.testing.assert_close(C.double(), Xg.double().t() @ G.double(), rtol=tol, atol=tol * 4)
    if ld == M:  # same operand layout -> same kernel and k order
        assert torch.equal(C, C2)


def _philox4x32_10(c, k):
    """Philox4x32-10 reference (numpy uint64 arithmetic), c: 4 x uint32 arrays, k: 2 ints."""
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    c = [x.astype(np.uint64) for x in c]
    k0, k1 = np.uint64(k[0]), np.uint64(k[1])
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(M0) * c[0]
        p1 = np.uint64(M1) * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & mask
        hi1, lo1 = p1 >> np.uint64(32), p1 & mask
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + np.uint64(W0)) & mask
        k1 = (k1 + np.uint64(W1)) & mask
    return [x.astype(np.uint32) for x in c]


def _dropout_keep(M, N, p, seed, offset):
    """Element (row, col): 16 bits of Philox4x32-10 at counter {row/4, col/2, offset}
    (word row % 4, low half for even col, high half for odd), kept iff >= floor(p * 2^16)."""
    rows = np.arange(M, dtype=np.uint64)[:, None] * np.ones((1, N), np.uint64)
    cols = np.ones((M, 1), np.uint64) * np.arange(N, dtype=np.uint64)[None, :]
    c = [(rows >> np.uint64(2)).astype(np.uint32), (cols >> np.uint64(1)).astype(np.uint32),
         np.full((M, N), offset & 0xFFFFFFFF, np.uint32), np.full((M, N), offset >> 32, np.uint32)]
    w = _philox4x32_10(c, (seed & 0xFFFFFFFF, seed >> 32))
    word = np.choose((rows & np.uint64(3)).astype(np.int64), w).astype(np.uint64)
    bits = np.where((cols & np.uint64(1)) == 1, word >> np.uint64(16), word & np.uint64(0xFFFF))
    thr = 65536 if p >= 1.0 else min(int(p * 65536.0), 65536)
    return bits >= np.uint64(thr)


@pytest.mark.parametrize("M,N,K,p", [(5000, 128, 602, 0.5), (333, 41, 100, 0.3), (1000, 128, 128, 0.0),
                                     (64, 7, 33, 1.0), (4001, 256, 128, 0.5), (2050, 64, 77, 0.2)])
def test_gemm_relu_dropout_epilogue(hip, M, N, K, p):
    """dropout(relu(A @ B)) fused in the GEMM epilogue: the mask is the
    documented Philox stream (checked against a numpy restatement), kept
    values are relu(AB)/(1-p) within fp32 GEMM tolerance."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.randn(M, K, device=DEV, generator=g)
    B = torch.randn(K, N, device=DEV, generator=g)
    C = torch.full((M, N), float("nan"), device=DEV)
    seed, offset = 0x1234_5678_9ABC, 77
    hip.gemm_relu_dropout(A, B, C, p=p, seed=seed, offset=offset)
    torch.cuda.synchronize()
    Z = (A.double() @ B.double()).cpu()
    keep = torch.from_numpy(_dropout_keep(M, N, p, seed, offset)) if p < 1.0 else torch.zeros(M, N, dtype=torch.bool)
    scale = 1.0 / (1.0 - p) if p < 1.0 else 0.0
    ref = torch.where(keep & (Z > 0), Z * scale, torch.zeros_like(Z))
    tol = 2e-6 * K ** 0.5 + 1e-6
    got = C.cpu().double()
    # elements whose relu decision sits within rounding of 0 may legitimately differ
    near0 = Z.abs() < 1e-4 * K ** 0.5
    torch.testing.assert_close(got[~near0], ref[~near0], rtol=tol, atol=tol * 4 * max(scale, 1))
    if 0 < p < 1:
        frac = keep.double().mean().item()
        assert abs(frac - (1 - p)) < 0.02
    # same (seed, offset) -> same output; another offset -> another mask
    C2 = torch.empty_like(C)
    hip.gemm_relu_dropout(A, B, C2, p=p, seed=seed, offset=offset)
    torch.cuda.synchronize()
    assert torch.equal(C, C2)


@pytest.mark.parametrize("M,N,K", [(602, 128, 20000), (128, 41, 3000), (64, 128, 77),
                                   (602, 128, 135758), (1000, 256, 999)])
def test_gemm_tn_masked(hip, M, N, K):
    """C = A^T (G * (X > 0) * scale): the relu+dropout backward fused into the
    weight-gradient GEMM."""
    g = torch.Generator(device=DEV).manual_seed(M * 3 + N + K)
    A = torch.randn(K, M, device=DEV, generator=g)
    G = torch.randn(K, N, device=DEV, generator=g)
    X = torch.relu(torch.randn(K, N, device=DEV, generator=g))
    C = torch.full((M, N), float("nan"), device=DEV)
    hip.gemm_tn_masked(A, G, X, C, scale=2.0)
    ref = A.double().t() @ (G.double() * (X > 0).double() * 2.0)
    torch.cuda.synchronize()
    tol = 2e-6 * K ** 0.5 + 1e-6
    torch.testing.assert_close(C.double(), ref, rtol=tol, atol=tol * 8)


@pytest.mark.parametrize("M,N,K,trans_a", [(136000, 128, 602, False), (4099, 256, 301, False),
                                           (602, 128, 20000, True), (333, 128, 777, True)])
def test_gemm_padded_pitch(hip, M, N, K, trans_a):
    """Row-padded operands (the bottom aggregation output has 128-byte aligned
    rows): the 16-byte A-load paths read the pitch, never the padding's values."""
    g = torch.Generator(device=DEV).manual_seed(M + K)
    rows, cols = (K, M) if trans_a else (M, K)
    ld = (cols + 31) // 32 * 32 + 32
    big = torch.full((rows, ld), float("nan"), device=DEV)
    A = big[:, :cols]
    A.copy_(torch.randn(rows, cols, device=DEV, generator=g))
    B = torch.randn(K, N, device=DEV, generator=g)
    C = torch.full((M, N), float("nan"), device=DEV)
    hip.gemm(A, B, C, trans_a=trans_a)
    ref = (A.double().t() if trans_a else A.double()) @ B.double()
    torch.cuda.synchronize()
    tol = 2e-6 * K ** 0.5 + 1e-6
    torch.testing.assert_close(C.double(), ref, rtol=tol, atol=tol * 4)
    C2 = torch.empty_like(C)
    hip.gemm(A.contiguous(), B, C2, trans_a=trans_a)
    torch.cuda.synchronize()
    torch.testing.assert_close(C2, C, rtol=tol, atol=tol * 4)


@pytest.mark.parametrize("n,K,C", [(10000, 128, 41), (1024, 256, 47), (33, 16, 7), (1, 16, 64),
                                   (5000, 128, 2), (77, 32, 17)])
def test_linear_xent_fused(hip, n, K, C):
    """Fused output layer + loss vs libtorch's own ops on the same tensors
    (Y @ W, log_softmax twice, mean nll_loss, autograd backward)."""
    g = torch.Generator(device=DEV).manual_seed(n + K + C)
    Y = torch.randn(n, K, device=DEV, generator=g)
    W = torch.randn(K, C, device=DEV, generator=g) * 0.1
    lab = torch.randint(0, C, (n,), device=DEV, generator=g)
    loss = torch.full((), float("nan"), device=DEV)
    correct = torch.full((1,), 5, dtype=torch.int32, device=DEV)
    hip.linear_xent_fwd(Y, W, lab, loss, correct)
    Yr, Wr = Y.double().requires_grad_(), W.double().requires_grad_()
    ref = torch.nn.functional.nll_loss((Yr @ Wr).log_softmax(1).log_softmax(1), lab)
    ref.backward(torch.tensor(1.7, dtype=torch.float64, device=DEV))
    torch.cuda.synchronize()
    torch.testing.assert_close(loss.double(), ref.detach(), rtol=1e-5, atol=1e-5)
    # getCorrect: argmax of log_softmax(Y W) == label, accumulated onto *correct
    # (fp32 logits: rows whose two best logits are within rounding may differ)
    z = (Y.double() @ W.double())
    top2 = z.topk(min(2, C), 1).values
    clear = (top2[:, 0] - top2[:, -1] > 1e-4) if C > 1 else torch.ones(n, dtype=torch.bool, device=DEV)
    want = int(((z.argmax(1) == lab) & clear).sum())
    unclear = int((~clear).sum())
    assert want <= int(correct) - 5 <= want + unclear
    dY = torch.full((n, K), float("nan"), device=DEV)
    dW = torch.full((K, C), float("nan"), device=DEV)
    gl = torch.tensor(1.7, device=DEV)
    hip.linear_xent_bwd(Y, W, lab, gl, dY, dW)
    torch.cuda.synchronize()
    torch.testing.assert_close(dY.double(), Yr.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(dW.double(), Wr.grad, rtol=1e-4, atol=1e-6)
    dY2, dW2, loss2 = torch.empty_like(dY), torch.empty_like(dW), torch.empty_like(loss)
    hip.linear_xent_fwd(Y, W, lab, loss2)
    hip.linear_xent_bwd(Y, W, lab, gl, dY2, dW2)
    torch.cuda.synchronize()
    assert torch.equal(loss, loss2) and torch.equal(dY, dY2) and torch.equal(dW, dW2)


@pytest.mark.gpu
@pytest.mark.parametrize("n,K,C,pad", [(10000, 128, 41, 0), (77, 32, 17, 3), (1, 16, 64, 0),
                                       (300, 256, 7, 4)])
def test_linear_xent_train(hip, n, K, C, pad):
    """The training call (loss + gradients for d loss = 1, one pass) is
    bit-identical to forward + backward(1), also on padded / unaligned rows
    (scalar staging path), and matches libtorch's autograd in fp64."""
    g = torch.Generator(device=DEV).manual_seed(3 * n + K + C)
    Yb = torch.randn(n, K + pad, device=DEV, generator=g)
    Y = Yb[:, :K]
    W = torch.randn(K, C, device=DEV, generator=g) * 0.1
    lab = torch.randint(0, C, (n,), device=DEV, generator=g)
    loss, loss2 = torch.full((), float("nan"), device=DEV), torch.full((), float("nan"), device=DEV)
    dY, dW = torch.full((n, K), float("nan"), device=DEV), torch.full((K, C), float("nan"), device=DEV)
    dY2, dW2 = torch.empty_like(dY), torch.empty_like(dW)
    for _ in range(2):  # the second call checks the loss ticket was reset
        hip.linear_xent_train(Y, W, lab, loss, dY, dW)
    hip.linear_xent_fwd(Y, W, lab, loss2)
    hip.linear_xent_bwd(Y, W, lab, torch.ones((), device=DEV), dY2, dW2)
    torch.cuda.synchronize()
    assert torch.equal(loss, loss2) and torch.equal(dY, dY2) and torch.equal(dW, dW2)
    Yr, Wr = Y.double().requires_grad_(), W.double().requires_grad_()
    ref = torch.nn.functional.nll_loss((Yr @ Wr).log_softmax(1).log_softmax(1), lab)
    ref.backward()
    torch.testing.assert_close(loss.double(), ref.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dY.double(), Yr.grad, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(dW.double(), Wr.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("rate", [0.0, 0.05, 0.37, 1.0])
@pytest.mark.parametrize("F", [41, 602])
def test_feature_cache_two_tier(hip, cora, rate, F):
    """HBM cache + host-pinned spill (GS_SAMPLE_PD_CACHE, load_feature_gpu_cache):
    the selection equals the oracle's degree order, and both the two-tier row
    gather and the fused two-tier aggregation are bit-identical to the
    full-table paths for every cache size."""
    from nts.hip import HostTable
    V, src, dst = cora
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    n_cache = int(round(rate * V))
    cmap = torch.empty(V, dtype=torch.int32, device=DEV)
    cids = torch.empty(max(n_cache, 1), dtype=torch.int32, device=DEV)
    hip.cache_select(g.out_degree, V, n_cache, cmap, cids if n_cache else None)
    torch.cuda.synchronize()
    cmap_ref, cids_ref = orc.cache_select(out_d, n_cache)
    assert np.array_equal(_np_u32(cmap), cmap_ref)
    assert np.array_equal(_np_u32(cids)[:n_cache], cids_ref)
    # host table with a 128-byte pitch (the bench layout), cache filled by gather_rows
    rng = np.random.default_rng(F + 1)
    table = rng.standard_normal((V, F)).astype(np.float32)
    ld = (F + 31) // 32 * 32
    host = HostTable(V, F, ld)
    host.tensor.copy_(torch.from_numpy(table))
    cache = None
    if n_cache:
        cache = torch.empty((n_cache, ld), device=DEV)[:, :F]
        nc = torch.tensor([n_cache], dtype=torch.int32, device=DEV)
        hip.gather_rows(_t(table), cids, nc, n_cache, cache)
    # sampled layers (PHILOX) and the reference values
    seeds = np.arange(0, V, 7, dtype=np.uint32)
    o = orc.Sampler(col, rows, in_d, out_d, [25, 10], rng_mode=orc.RNG_PHILOX,
                    order_mode=orc.ORDER_DRAW)
    l0, l1 = o.sample(seeds)
    X = orc.get_feature(l1["source"], table)
    Y_ref = orc.fuse_fwd(l1, X, out_d, in_d)
    s, v = l1["src_size"], l1["v_size"]
    # two-tier row gather == get_feature (== the oracle's two-tier restatement)
    x0 = torch.full((s, F), float("nan"), device=DEV)
    n = torch.tensor([s], dtype=torch.int32, device=DEV)
    hip.gather_rows_cached(cache, cmap, host, _t(l1["source"]), n, s, x0)
    # fused two-tier aggregation == MiniBatchFuseOp::forward
    co, ri, wf = _t(l1["column_offset"]), _t(l1["row_indices"]), _t(l1["edge_weight_forward"])
    vdev = torch.tensor([v], dtype=torch.int32, device=DEV)
    y = torch.full((v, ld), 5.0, device=DEV)
    hip.spmm_csc_fwd_cached(co, ri, wf, vdev, v, cache, cmap, host, _t(l1["source"]), y[:, :F])
    torch.cuda.synchronize()
    assert np.array_equal(x0.cpu().numpy(), X)
    if n_cache:
        assert np.array_equal(
            orc.get_feature_cached(l1["source"], cache.cpu().numpy(), cmap_ref, table), X)
    assert np.array_equal(y[:, :F].cpu().numpy(), Y_ref)
    assert (y[:, F:] == 5.0).all()
    # spilled rows staged once per batch by local id, then the fused aggregation
    stage = torch.full((s, ld), float("nan"), device=DEV)
    hip.stage_uncached_rows(cmap, host, _t(l1["source"]), n, s, stage[:, :F])
    y2 = torch.empty((v, F), device=DEV)
    hip.spmm_csc_fwd_cached(co, ri, wf, vdev, v, cache, cmap, host, _t(l1["source"]), y2,
                            stage=stage[:, :F])
    torch.cuda.synchronize()
    cold = cmap_ref[l1["source"]] == orc.NOT_CACHED
    st = stage[:, :F].cpu().numpy()
    assert np.array_equal(st[cold], X[cold])
    assert np.isnan(st[~cold]).all()  # cached rows are never staged
    assert np.array_equal(y2.cpu().numpy(), Y_ref)
    host.close()


def _gat_torch(H, att, co, ri, dl, F):
    """The reference layer chain (GAT_SAMPLE_ALL_GPU.hpp:354-388) in torch fp64 with
    materialised messages: msg = [H[src], H[dst]], m = leaky(msg W_att), per-dst
    softmax (max-subtracted, edge_softmax_forward_norm_block), sum a*H[src], relu."""
    v = co.numel() - 1
    deg = (co[1:] - co[:-1]).long()
    d_of_e = torch.repeat_interleave(torch.arange(v, device=H.device), deg)
    msg = torch.cat([H[ri.long()], H[dl.long()[d_of_e]]], 1)
    m = torch.nn.functional.leaky_relu(msg @ att.view(2 * F, 1), 0.2).view(-1)
    mx = torch.full((v,), -float("inf"), dtype=H.dtype, device=H.device).scatter_reduce(
        0, d_of_e, m, "amax")
    ex = torch.exp(m - mx[d_of_e])
    sm = torch.zeros(v, dtype=H.dtype, device=H.device).index_add(0, d_of_e, ex)
    a = ex / sm[d_of_e]
    Z = torch.zeros(v, F, dtype=H.dtype, device=H.device).index_add(0, d_of_e, H[ri.long()] * a[:, None])
    return torch.relu(Z), m, a


@pytest.mark.parametrize("F", [16, 7, 256])
def test_gat_layer_matches_torch(hip, cora, F):
    """Fused GAT layer (forward: online softmax; backward: per-dst + CSR passes)
    vs autograd through the reference's materialised-message chain, fp64."""
    V, src, dst = cora
    g = _graph(hip, V, src, dst)
    seeds = np.arange(0, V, 9, dtype=np.uint32)
    lays = _sample_gpu(hip, g, seeds, [10, 5], 0, 1, 0, merge=True)
    lay = lays[1]
    v, e, s, _ = lay.sizes_host()
    gen = torch.Generator(device=DEV).manual_seed(F)
    H = torch.randn(s, F, device=DEV, generator=gen)
    att = torch.randn(2 * F, device=DEV, generator=gen) * 0.3
    co, ri, dl = lay.column_offset[:v + 1], lay.row_indices[:e], lay.dst_local_id[:v]
    m = torch.empty(e, device=DEV)
    a = torch.empty(e, device=DEV)
    Y = torch.empty(v, F, device=DEV)
    hip.gat_forward(co, ri, dl, v, H, att, m, a, Y)
    Hd = H.double().requires_grad_(True)
    attd = att.double().requires_grad_(True)
    Yr, mr, ar = _gat_torch(Hd, attd, co, ri, dl, F)
    torch.testing.assert_close(Y.double(), Yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(m.double(), mr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(a.double(), ar, rtol=1e-5, atol=1e-6)
    GY = torch.randn(v, F, device=DEV, generator=gen)
    Yr.backward(GY.double())
    du = torch.empty(e, device=DEV)
    ds2 = torch.empty(s, device=DEV)
    dH = torch.empty(s, F, device=DEV)
    dS = torch.empty(s, 2, device=DEV)
    hip.gat_backward(co, ri, dl, v, lay.row_offset, lay.column_indices, lay.csr_edge_id, s, H, att,
                     a, m, Y, GY, du, ds2, dH, dS)
    torch.cuda.synchronize()
    torch.testing.assert_close(dH.double(), Hd.grad, rtol=1e-4, atol=1e-5)
    datt = torch.cat([H.double().t() @ dS[:, 0].double(), H.double().t() @ dS[:, 1].double()])
    torch.testing.assert_close(datt, attd.grad, rtol=1e-4, atol=1e-4)
    # deterministic: a second backward is bit-identical
    dH2 = torch.empty_like(dH)
    hip.gat_backward(co, ri, dl, v, lay.row_offset, lay.column_indices, lay.csr_edge_id, s, H, att,
                     a, m, Y, GY, du, ds2, dH2, dS)
    torch.cuda.synchronize()
    assert torch.equal(dH, dH2)


@pytest.mark.parametrize("F,mask", [(128, False), (128, True), (256, False), (602, False), (7, True)])
def test_csr_bwd_long_rows_cooperative(hip, F, mask):
    """A hub sampled by thousands of destinations gives one CSR row of thousands
    of edges (the power-law case): summed by the whole workgroup in GPB in-order
    pieces — deterministic run to run and equal to the fp64 sum within fp32
    rounding; short rows stay bit-exact."""
    rng = np.random.default_rng(F)
    s, v = 300, 5000
    # CSR rows: row 0 (the hub) gets 4000 edges, row 1 2000, the rest 0..6 each
    lens = np.concatenate([[4000, 2000], rng.integers(0, 7, s - 2)])
    ro = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
    e = int(ro[-1])
    ci = rng.integers(0, v, e).astype(np.uint32)
    wb = rng.random(e).astype(np.float32)
    G = rng.standard_normal((v, F)).astype(np.float32)
    Xa = np.maximum(rng.standard_normal((v, F)).astype(np.float32), 0)
    Gm = np.where(Xa > 0, G * np.float32(2), np.float32(0)).astype(np.float32) if mask else G
    ref = np.zeros((s, F), np.float64)
    for r in range(s):
        for j in range(ro[r], ro[r + 1]):
            ref[r] += np.float64(wb[j]) * Gm[ci[j]].astype(np.float64)
    outs = []
    for _ in range(2):
        gin = torch.empty(s, F, device=DEV)
        if mask:
            hip.spmm_csr_bwd_masked(_t(ro), _t(ci), _t(wb), None, s, _t(G), _t(Xa), gin, scale=2.0)
        else:
            hip.spmm_csr_bwd(_t(ro), _t(ci), _t(wb), None, s, _t(G), gin)
        torch.cuda.synchronize()
        outs.append(gin.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    np.testing.assert_allclose(outs[0], ref, rtol=2e-5, atol=2e-4)
    # short rows: the serial edge order exactly
    for r in range(2, s):
        acc = np.zeros(F, np.float32)
        for j in range(ro[r], ro[r + 1]):
            acc = acc + Gm[ci[j]] * wb[j]
        assert np.array_equal(outs[0][r], acc)


@pytest.mark.parametrize("rows,F,pad", [(1000, 128, False), (333, 41, False), (77, 7, True)])
def test_act_backward(hip, rows, F, pad):
    """dZ = dX * [X > 0] * scale; + the plain CSR gather == the masked gather."""
    g = torch.Generator(device=DEV).manual_seed(rows)
    ld = F + 5 if pad else F
    G = torch.randn(rows, ld, device=DEV, generator=g)[:, :F]
    X = torch.relu(torch.randn(rows, ld, device=DEV, generator=g))[:, :F]
    out = torch.full((rows, ld), float("nan"), device=DEV)[:, :F]
    hip.act_backward(G, X, out, scale=2.0)
    torch.cuda.synchronize()
    ref = torch.where(X > 0, G * 2.0, torch.zeros_like(G))
    assert torch.equal(out, ref)


@pytest.mark.parametrize("rng_mode", [0])
def test_capacity_overflow_flag_survives_multi_tile_scan(hip, rng_mode):
    """The fused count scan sets the overflow flag from ONE thread (the item
    at n), for the edge capacity and the dst capacity alike, with the dsts
    spanning several 4,096-item scan tiles: a truncated layer is always
    reported (a block-0 clear racing an atomicOr from another
    tile could lose it)."""
    from nts.hip import LayerBuffers
    V, src, dst = _random_graph(30000, 600000, 11)
    g = _graph(hip, V, src, dst)
    seeds = np.arange(0, 14000, dtype=np.uint32)  # 4 scan tiles
    hip.reserve(V, 14000 * 10)
    dst_t = _t(seeds)
    vsz = torch.tensor([seeds.size], dtype=torch.int32, device=DEV)
    for rep in range(8):
        # edge capacity exceeded
        lay = LayerBuffers(14000, 5000, 14000 * 10, dst_t, vsz, torch.device(DEV))
        hip.sample_layer(g, lay, 10, 0, rep, rng_mode, 0)
        torch.cuda.synchronize()
        v, e, s, ovf = lay.sizes_host()
        assert v == 14000 and 0 < e <= 5000 and (ovf & 1), (rep, v, e, ovf)
        # truncated at a destination boundary: every edge slot below e_size
        # was written (valid ids), and e_size is one of the column offsets
        co = _np_u32(lay.column_offset)[:v + 1]
        assert e in set(co.tolist())
        assert (_np_u32(lay.sample_ans)[:e] < V).all() and (_np_u32(lay.row_indices)[:e] < s).all()
        # dst capacity exceeded (v_req = 14000 > v_cap = 9000)
        lay = LayerBuffers(9000, 9000 * 10, 9000 * 10, dst_t, vsz, torch.device(DEV))
        hip.sample_layer(g, lay, 10, 0, rep, rng_mode, 0)
        torch.cuda.synchronize()
        v, e, s, ovf = lay.sizes_host()
        assert v == 9000 and (ovf & 1), (rep, v, e, ovf)
        # in capacity: no flag
        lay = LayerBuffers(14000, 14000 * 10, 14000 * 10, dst_t, vsz, torch.device(DEV))
        hip.sample_layer(g, lay, 10, 0, rep, rng_mode, 0)
        torch.cuda.synchronize()
        assert lay.sizes_host()[3] == 0


@pytest.mark.parametrize("V", [1500, 100_000, 400_000, 600_000])
def test_csr_transpose_bucket_geometries(hip, V):
    """The CSR transpose (round 6: one radix pass on the high H source bits +
    k_csr_bucket per 2^L sources) at every bucket geometry — 11-bit source
    ids (H = 5, L = 6), 17 (9, 8), 19 (9, 10: 1,024-row buckets) and 20 bits
    (past the bucket form: the two-pass sort + k_csr_finalize) — on a graph
    with a hub source every dst links to (one CSR row spread over every wave
    of its bucket): all arrays bit-exact vs the oracle's serial fill."""
    src, dst = _random_graph(V, 8 * V, V)[1:]
    hub = np.arange(1, V, dtype=np.uint32)
    src = np.concatenate([src, np.zeros(V - 1, np.uint32)])
    dst = np.concatenate([dst, hub])
    g = _graph(hip, V, src, dst)
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    seeds = np.random.default_rng(V).choice(V, V // 10, replace=False).astype(np.uint32)
    o = orc.Sampler(col, rows, in_d, out_d, [10], seed=2000, rng_mode=orc.RNG_PHILOX,
                    order_mode=orc.ORDER_DRAW)
    gl = [_gpu_layer_np(l) for l in _sample_gpu(hip, g, seeds, [10], 0, 1, 1)]
    ol = o.sample(seeds, 1, 1)
    assert ol[0]["src_size"] > 100
    _assert_layers_equal(gl, ol)
