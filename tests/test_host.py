"""End-to-end parity of the C++ host layer (FastSampler, SingleGPUAllSampleGraphOp,
NtsContext, Parameter, GCN driver) against the CPU oracle of the reference's
GCN_CPU_SAMPLE path.

Bars: sampled structures bit-exact; forward activations within 1e-4 (fp32;
the aggregation outputs themselves are bit-exact); one full training step
(backward through the context + Adam) within 1e-5 of the oracle.
"""
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


@pytest.fixture(scope="module")
def graph(E):
    from nts import synthetic
    g = synthetic.chung_lu(6000, 180000, 20.0, device=DEV, seed=3)
    G = E.FullyRepGraph.from_edges(g.src, g.dst, g.n_vertices)
    src = g.src.cpu().numpy().view(np.uint32)
    dst = g.dst.cpu().numpy().view(np.uint32)
    col, rows = orc.build_csc(g.n_vertices, src, dst)
    od, idg = orc.degrees(g.n_vertices, src, dst)
    return dict(G=G, V=g.n_vertices, col=col, rows=rows, od=od, idg=idg)


def _np(t):
    a = t.cpu().numpy()
    return a.view(np.uint32) if a.dtype == np.int32 else a


def test_fast_sampler_matches_oracle(E, graph):
    seeds = torch.arange(0, 3000, 2, dtype=torch.int32)
    fs = E.FastSampler(graph["G"], seeds, 2, 500, [25, 10])
    o = orc.Sampler(graph["col"], graph["rows"], graph["idg"], graph["od"], [25, 10],
                    rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    bs = 0
    while fs.sample_not_finished():
        got = fs.sample_gpu_fast(500)
        ref = o.sample(seeds.numpy()[bs * 500:(bs + 1) * 500].astype(np.uint32), bs)
        for a, b in zip(got, ref):
            assert (a["v_size"], a["e_size"], a["src_size"]) == (b["v_size"], b["e_size"], b["src_size"])
            for k in ("destination", "column_offset", "row_indices", "sample_ans", "source",
                      "edge_weight_forward", "row_offset", "column_indices", "edge_weight_backward"):
                assert np.array_equal(_np(a[k]), b[k]), k
        bs += 1
    assert bs == 3


def _driver(E, graph, F, C, layers, fanout, batch, drop=0.0, seed=2000, comm=None, **kw):
    from nts import host, synthetic
    feat = synthetic.features(graph["V"], F, device=DEV)
    labels, masks = synthetic.labels_masks(graph["V"], C, device=DEV)
    train = torch.nonzero(masks == 0).flatten().to(torch.int32).cpu()
    cfg = host.gcn_config(layers, fanout, batch, learn_rate=0.01, drop_rate=drop, seed=seed,
                          shuffle=False, **kw)
    drv = E.GCN_SAMPLE_ALLGPU_impl(graph["G"], feat, labels, train, cfg, comm)
    return drv, feat, labels, train


@pytest.mark.parametrize("F,tf,pt", [(602, 0, 1), (128, 0, 1), (602, 1, 0), (602, 1, 1),
                                     (128, 1, 2), (48, 1, 1), (602, 1, 3)])
def test_gcn_forward_activations_match_gcn_cpu_sample(E, graph, F, tf, pt):
    """tf = 0: aggregate first, the reference's order (Y0 bit-exact);
    tf = 1: transform first, A (X W0): H = X W0 and every later activation
    within the north-star's 1e-4 of the GCN_CPU_SAMPLE chain (pt: the
    forward GEMM on the fp32 table (0) or on its f16 pair table (1, 2))."""
    H = 128 if pt == 3 else 64
    drv, feat, labels, _ = _driver(E, graph, F, 41, [F, H, 41], [25, 10], 256, transform_first=tf,
                                   pair_table=pt)
    assert drv.transform_first == bool(tf)
    seeds = torch.arange(7, 7 + 256, dtype=torch.int32)
    acts = drv.forward_eval(seeds, 3)
    W = [w.cpu() for w in drv.weights()]
    o = orc.Sampler(graph["col"], graph["rows"], graph["idg"], graph["od"], [25, 10],
                    rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, l1 = o.sample(seeds.numpy().astype(np.uint32), 3)
    # GCN_CPU_SAMPLE forward (toolkits/GCN_CPU_SAMPLE.hpp:214-233), eval mode
    X0 = orc.get_feature(l1["source"], feat.cpu().numpy())
    Y0 = orc.fuse_fwd(l1, X0, graph["od"], graph["idg"])
    X1 = torch.relu(torch.from_numpy(Y0) @ W[0])
    Y1 = orc.fuse_fwd(l0, X1.numpy(), graph["od"], graph["idg"])
    X2 = (torch.from_numpy(Y1) @ W[1]).log_softmax(1)
    if tf:
        H = torch.from_numpy(X0).double() @ W[0].double()
        torch.testing.assert_close(acts[0].cpu().double(), H, rtol=1e-5, atol=1e-5)
    else:
        assert np.array_equal(acts[0].cpu().numpy(), Y0)  # fused gather+aggregation: bit-exact
    torch.testing.assert_close(acts[1].cpu(), X1, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(acts[2].cpu(), torch.from_numpy(Y1), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(acts[3].cpu(), X2, rtol=1e-4, atol=1e-4)


def test_unfused_gather_path_is_identical(E, graph):
    from nts import host
    drv, feat, labels, train = _driver(E, graph, 96, 7, [96, 32, 7], [10, 5], 128, transform_first=0)
    cfg = host.gcn_config([96, 32, 7], [10, 5], 128, drop_rate=0.0, fused_gather=False,
                          shuffle=False, transform_first=0)
    drv2 = E.GCN_SAMPLE_ALLGPU_impl(graph["G"], feat, labels, train, cfg)
    drv2.set_weights(drv.weights())
    seeds = torch.arange(100, 228, dtype=torch.int32)
    a = drv.forward_eval(seeds, 0)   # gather fused into the graph op
    b = drv2.forward_eval(seeds, 0)  # load_feature_gpu, then the graph op
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("drop", [0.0, 0.5])
def test_transform_first_trains_like_aggregate_first(E, graph, drop):
    """A (X W) vs (A X) W: the same sampled batches and dropout masks (the
    aggregation epilogue uses the GEMM epilogue's keys), so one training step
    agrees to fp32 summation order (loss, weights after Adam)."""
    a, *_ = _driver(E, graph, 96, 7, [96, 32, 7], [10, 5], 200, drop=drop, transform_first=1)
    b, *_ = _driver(E, graph, 96, 7, [96, 32, 7], [10, 5], 200, drop=drop, transform_first=0)
    assert a.transform_first and not b.transform_first
    b.set_weights(a.weights())
    a.train_batch()
    b.train_batch()
    a.synchronize()
    b.synchronize()
    torch.testing.assert_close(a.loss, b.loss, rtol=1e-5, atol=1e-6)
    for x, y in zip(a.weights(), b.weights()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("overlap,tf", [(0, 0), (1, 0), (1, 1)])
def test_one_rank_communicator_is_identical(E, graph, overlap, tf):
    """The C++ data-parallel path on one GPU: initial ncclBroadcast of the
    weights, the fused gradient bucket (pack -> ncclAllReduce SUM -> unpack)
    every step (GCN_SAMPLE_ALL_MULTI::Update, toolkits/GCN_SAMPLE_ALL_MULTI.hpp:367-377);
    overlap = 1: the all-reduce on its own stream with the optimizer step
    deferred past the next batch's bottom aggregation.  At one rank the sum
    is the identity: bit-identical weights to comm=None."""
    comm = E.Communicator(1, 0, E.Communicator.unique_id(), 0)
    assert comm.nranks == 1
    a, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, drop=0.5, comm=comm,
                    overlap_allreduce=overlap, transform_first=tf)
    b, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, drop=0.5, transform_first=tf)
    for _ in range(5):
        a.train_batch()
        b.train_batch()
    a.synchronize()
    b.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        assert torch.equal(x, y)


@pytest.mark.parametrize("tf,pt", [(0, 1), (1, 0), (1, 1), (1, 2), (1, 3), (0, 3)])
def test_training_step_matches_oracle_step(E, graph, tf, pt):
    """One train_batch: sample -> forward -> NLL -> self_backward (graph-op
    backward through the CSR) -> learn_local_with_decay_Adam, vs the oracle
    (tf = 1: the bottom layer transform-first, its backward through the bottom
    layer's CSR and the row-gathered weight-gradient GEMM; tf = 0, H 128: the
    narrow aggregate-first bottom layer's forward on the in-kernel pair
    split, nts_hip_gemm_h2d_act)."""
    F, C, B = 64, 7, 200
    H = 128 if pt == 3 else 32  # pt 3: the planar weight-gradient kernel takes N % 128 == 0
    drv, feat, labels, train = _driver(E, graph, F, C, [F, H, C], [10, 5], B, transform_first=tf,
                                       pair_table=pt)
    W0 = [w.cpu().clone() for w in drv.weights()]
    drv.train_batch()
    drv.synchronize()
    W1 = [w.cpu() for w in drv.weights()]
    # oracle: same seeds (no shuffle), batch_seq 0, PHILOX stream
    seeds = train.numpy()[:B].astype(np.uint32)
    o = orc.Sampler(graph["col"], graph["rows"], graph["idg"], graph["od"], [10, 5],
                    rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, l1 = o.sample(seeds, 0)
    W = [w.clone().requires_grad_() for w in W0]
    X0 = orc.get_feature(l1["source"], feat.cpu().numpy())
    Y0 = torch.from_numpy(orc.fuse_fwd(l1, X0, graph["od"], graph["idg"]))
    X1 = torch.relu(Y0 @ W[0])
    Y1 = torch.from_numpy(orc.fuse_fwd(l0, X1.detach().numpy(), graph["od"], graph["idg"])).requires_grad_()
    X2 = (Y1 @ W[1]).log_softmax(1)
    tgt = labels.cpu()[torch.from_numpy(l0["destination"].astype(np.int64))]
    loss = torch.nn.functional.nll_loss(X2.log_softmax(1), tgt)
    loss.backward()
    gX1 = orc.fuse_bwd(l0, Y1.grad.numpy(), graph["od"], graph["idg"])
    X1.backward(torch.from_numpy(gX1))
    for w0, w, w1 in zip(W0, W, W1):
        g = w.grad
        wg = w0 * 1e-4 + g
        m = 0.1 * wg
        v = (0.001 * wg) * wg
        ref = w0 - (0.01 * m) / (torch.sqrt(v) + 1e-9)
        torch.testing.assert_close(w1, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("tf", [0, 1])
def test_atomic_backward_trains_like_the_csr_backward(E, graph, tf):
    """deterministic_backward=False (graph-op backward by atomic CSC scatter,
    no CSR in the sampler) — with the transform-first bottom layer too, where
    the layer above then has no CSR to fuse the activation backward into:
    the same step as the CSR-gather backward, up to fp32 summation order."""
    a, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, drop=0.5, transform_first=tf,
                    deterministic_backward=False)
    b, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, drop=0.5, transform_first=tf)
    assert a.transform_first == bool(tf)
    for _ in range(2):
        a.train_batch()
        b.train_batch()
    a.synchronize()
    b.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-4)


def _gcn_cpu_sample_forward(graph, feat, W, l0, l1):
    """GCN_CPU_SAMPLE forward (toolkits/GCN_CPU_SAMPLE.hpp:214-233), eval mode."""
    X0 = orc.get_feature(l1["source"], feat.cpu().numpy())
    Y0 = orc.fuse_fwd(l1, X0, graph["od"], graph["idg"])
    X1 = torch.relu(torch.from_numpy(Y0) @ W[0])
    Y1 = orc.fuse_fwd(l0, X1.numpy(), graph["od"], graph["idg"])
    X2 = (torch.from_numpy(Y1) @ W[1]).log_softmax(1)
    return [torch.from_numpy(Y0), X1, torch.from_numpy(Y1), X2]


@pytest.mark.parametrize("tf", [0, 1])
def test_gcn_sample_gpu_reference_stream(E, graph, tf):
    """GCN_SAMPLE_GPU (toolkits/GCN_SAMPLE_GPU.hpp:289-394): blocks of the
    reference's own sampler stream (sample_fast, std::mt19937(2000), replayed
    on the device) through SingleGPUSampleGraphOp (CSR backward).  Forward
    activations vs the GCN_CPU_SAMPLE chain on the oracle's blocks in the
    reference's own emission order (std::unordered_map per dst) within the
    north star's 1e-4; then one training step vs the oracle's step."""
    from nts import _abi
    F, C, B = 96, 7, 200
    kw = dict(rng_mode=_abi.NTS_RNG_MT19937_LEMIRE, sample_gpu=True, transform_first=tf)
    drv, feat, labels, train = _driver(E, graph, F, C, [F, 32, C], [10, 5], B, **kw)
    seeds = torch.arange(11, 11 + 256, dtype=torch.int32)
    acts = drv.forward_eval(seeds, 0)
    W = [w.cpu() for w in drv.weights()]
    o = orc.Sampler(graph["col"], graph["rows"], graph["idg"], graph["od"], [10, 5], seed=2000,
                    rng_mode=orc.RNG_MT_LEMIRE, order_mode=orc.ORDER_UNORDERED_MAP)
    l0, l1 = o.sample(seeds.numpy().astype(np.uint32), 0)
    ref = _gcn_cpu_sample_forward(graph, feat, W, l0, l1)
    for got, r in zip(acts[1:], ref[1:]):
        torch.testing.assert_close(got.cpu(), r, rtol=1e-4, atol=1e-4)
    if not tf:
        torch.testing.assert_close(acts[0].cpu(), ref[0], rtol=1e-5, atol=1e-6)
    # one training step on a fresh driver (fresh generator) vs the oracle
    drv, feat, labels, train = _driver(E, graph, F, C, [F, 32, C], [10, 5], B, **kw)
    W0 = [w.cpu().clone() for w in drv.weights()]
    drv.train_batch()
    drv.synchronize()
    W1 = [w.cpu() for w in drv.weights()]
    o = orc.Sampler(graph["col"], graph["rows"], graph["idg"], graph["od"], [10, 5], seed=2000,
                    rng_mode=orc.RNG_MT_LEMIRE, order_mode=orc.ORDER_UNORDERED_MAP)
    l0, l1 = o.sample(train.numpy()[:B].astype(np.uint32), 0)
    Wg = [w.clone().requires_grad_() for w in W0]
    X0 = orc.get_feature(l1["source"], feat.cpu().numpy())
    Y0 = torch.from_numpy(orc.fuse_fwd(l1, X0, graph["od"], graph["idg"]))
    X1 = torch.relu(Y0 @ Wg[0])
    Y1 = torch.from_numpy(orc.fuse_fwd(l0, X1.detach().numpy(), graph["od"],
                                       graph["idg"])).requires_grad_()
    X2 = (Y1 @ Wg[1]).log_softmax(1)
    tgt = labels.cpu()[torch.from_numpy(l0["destination"].astype(np.int64))]
    torch.nn.functional.nll_loss(X2.log_softmax(1), tgt).backward()
    X1.backward(torch.from_numpy(orc.fuse_bwd(l0, Y1.grad.numpy(), graph["od"], graph["idg"])))
    for w0, w, w1 in zip(W0, Wg, W1):
        wg = w0 * 1e-4 + w.grad
        ref_w = w0 - (0.01 * (0.1 * wg)) / (torch.sqrt((0.001 * wg) * wg) + 1e-9)
        torch.testing.assert_close(w1, ref_w, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("drop", [0.0, 0.5])
def test_training_is_deterministic_and_learns(E, graph, drop):
    a, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, drop=drop)
    b, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, drop=drop)
    for _ in range(2):
        a.run_epoch()
        b.run_epoch()
    a.synchronize()
    b.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        assert torch.equal(x, y)
    assert torch.isfinite(a.loss).item()


def test_early_aggregation_is_identical(E, graph):
    """Bottom graph op issued behind the sampler (early_aggregate) vs inside the
    forward: same sampled graphs, same kernels -> identical weights."""
    a, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, early_aggregate=True,
                    transform_first=0)
    b, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, early_aggregate=False,
                    transform_first=0)
    for _ in range(3):
        a.train_batch()
        b.train_batch()
    a.synchronize()
    b.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        assert torch.equal(x, y)


def test_fused_activation_matches_torch_ops(E, graph):
    """relu (+ dropout at p = 0) in the GEMM epilogue and its backward in the
    weight-gradient GEMM vs torch relu/dropout around the plain GEMM."""
    a, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, fuse_activation=True,
                    transform_first=0)
    b, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, fuse_activation=False)
    for _ in range(3):
        a.train_batch()
        b.train_batch()
    a.synchronize()
    b.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("rate", [0.0, 0.25, 1.0])
@pytest.mark.parametrize("early,fused", [(False, True), (True, True), (False, False)])
def test_feature_cache_training_is_identical(E, graph, rate, early, fused):
    """Features in pinned host memory with the highest-degree rows cached in
    HBM (GS_SAMPLE_PD_CACHE placement, cache_rate) train to the same weights
    as the all-HBM table: the two-tier reads change where rows come from, not
    their values (fused graph op, early aggregation, and load_feature_gpu_cache)."""
    kw = dict(early_aggregate=early, fused_gather=fused, transform_first=0)
    a, *_ = _driver(E, graph, 602, 7, [602, 32, 7], [10, 5], 200, drop=0.5, **kw)
    b, *_ = _driver(E, graph, 602, 7, [602, 32, 7], [10, 5], 200, drop=0.5, cache_rate=rate, **kw)
    for _ in range(3):
        a.train_batch()
        b.train_batch()
    a.synchronize()
    b.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        assert torch.equal(x, y)


def test_pipeline_carries_batches_across_passes(E, graph):
    """The pipelined driver samples the next pass's first batch behind the
    current pass's last one (no drain at pass boundaries); the batch sequence,
    and so the trained weights, equal the unpipelined driver's over several
    passes mixed with restart() calls."""
    a, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 300, drop=0.5, pipeline=True)
    b, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 300, drop=0.5, pipeline=False)
    for d in (a, b):
        d.run_epoch()
        d.restart()
        d.restart()  # repeated restarts without training in between are no-ops
        d.run_epoch()
        for _ in range(3):  # bench-style stepping across a pass boundary
            if not d.sample_not_finished():
                d.restart()
            d.train_batch()
        d.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        assert torch.equal(x, y)


@pytest.mark.parametrize("gate", [1, 2])
def test_sampler_gate_trains_identically(E, graph, gate):
    """--sampler-gate only moves where the next batch's sampling is issued
    (behind the transform-first bottom forward GEMM; with 2 the backward GEMM
    also waits for it): weights bit-identical to the ungated pipeline across
    pass boundaries."""
    a, *_ = _driver(E, graph, 602, 7, [602, 32, 7], [10, 5], 300, drop=0.5, pipeline=True,
                    transform_first=1, sampler_gate=gate)
    b, *_ = _driver(E, graph, 602, 7, [602, 32, 7], [10, 5], 300, drop=0.5, pipeline=True,
                    transform_first=1)
    for d in (a, b):
        d.run_epoch()
        for _ in range(3):
            if not d.sample_not_finished():
                d.restart()
            d.train_batch()
        d.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        assert torch.equal(x, y)


def _gat_layer_ref(X, W, att, ly):
    """GAT_SAMPLE_ALL_GPU layer (toolkits/GAT_SAMPLE_ALL_GPU.hpp:322-388), fp64,
    materialised messages, on an oracle-sampled merged layer."""
    H = X @ W
    F = W.shape[1]
    co = torch.from_numpy(ly["column_offset"].astype(np.int64))
    ri = torch.from_numpy(ly["row_indices"].astype(np.int64))
    dl = torch.from_numpy(ly["dst_local_id"].astype(np.int64))
    v = co.numel() - 1
    d_of_e = torch.repeat_interleave(torch.arange(v), co[1:] - co[:-1])
    msg = torch.cat([H[ri], H[dl[d_of_e]]], 1)
    m = torch.nn.functional.leaky_relu(msg @ att.view(2 * F, 1), 0.2).view(-1)
    mx = torch.full((v,), -float("inf"), dtype=H.dtype).scatter_reduce(0, d_of_e, m, "amax")
    ex = torch.exp(m - mx[d_of_e])
    a = ex / torch.zeros(v, dtype=H.dtype).index_add(0, d_of_e, ex)[d_of_e]
    Z = torch.zeros(v, F, dtype=H.dtype).index_add(0, d_of_e, H[ri] * a[:, None])
    return torch.relu(Z)


def test_gat_forward_matches_reference_chain(E, graph):
    drv, feat, labels, _ = _driver(E, graph, 96, 7, [96, 32, 7], [10, 5], 200, gat=True)
    seeds = torch.arange(11, 211, dtype=torch.int32)
    acts = drv.forward_eval(seeds, 5)
    W = [w.cpu().double() for w in drv.weights()]
    o = orc.Sampler(graph["col"], graph["rows"], graph["idg"], graph["od"], [10, 5],
                    rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, l1 = o.sample(seeds.numpy().astype(np.uint32), 5, orc.W_NONE | orc.F_MERGE_SRC_DST)
    X = torch.from_numpy(feat.cpu().numpy()[l1["source"]]).double()
    X1 = _gat_layer_ref(X, W[0], W[1], l1)
    X2 = _gat_layer_ref(X1, W[2], W[3], l0)
    torch.testing.assert_close(acts[0].cpu().double(), X1, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(acts[1].cpu().double(), X2, rtol=1e-4, atol=1e-5)


def test_gat_training_deterministic_and_learns(E, graph):
    a, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, gat=True, pipeline=True)
    b, *_ = _driver(E, graph, 64, 7, [64, 32, 7], [10, 5], 200, gat=True, pipeline=False)
    losses = []
    for _ in range(3):
        a.run_epoch()
        b.run_epoch()
        losses.append(float(a.loss.detach()))
    a.synchronize()
    b.synchronize()
    for x, y in zip(a.weights(), b.weights()):
        assert torch.equal(x, y)
    assert all(np.isfinite(losses))


def test_last_layers_is_the_trained_batch_across_a_partial_batch(E, graph):
    """bench.py reads last_layers after the timed steps; with the pipeline the
    sampler's current slot already holds the next (possibly partial) batch.
    last_layers must describe the batch just trained, whatever its size."""
    drv, _, _, train = _driver(E, graph, 32, 5, [32, 16, 5], [10, 5], 1000)
    n = int(train.numel())
    sizes = [min(1000, n - 1000 * b) for b in range((n + 999) // 1000)]
    assert sizes[-1] < 1000  # the pass ends with a partial batch
    for step in range(2 * len(sizes) + 1):
        if not drv.sample_not_finished():
            drv.restart()
        drv.train_batch()
        lay = drv.last_layers
        assert lay[0]["v_size"] == sizes[step % len(sizes)]
        assert lay[0]["destination"].numel() == lay[0]["v_size"]
    drv.synchronize()
