"""Pin the CPU oracle (oracle/ref_cpu.cpp) before trusting it.

The reference ships no tests or golden vectors and may not be
built or run here, so the oracle is pinned by:
  * known-answer tests independent of the RNG (hand-computed 5-vertex graph,
    fanout >= max degree -> full neighbourhoods, all-ones features ->
    row sums of the weights),
  * an independent restatement of the reference's RNG consumption
    (numpy's MT19937 with std::mt19937's init_genrand seeding + a Python
    Lemire draw + set semantics) that must reproduce the oracle's neighbour
    sets on the reference's own Cora graph (tests/golden/cora),
  * numpy float32 restatements of the aggregation arithmetic.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from nts import dataloader
from conftest import GOLDEN

# ---------------------------------------------------------------------------
# hand-computed 5-vertex graph
#   edges (src -> dst), file order:
#   0->1, 2->1, 1->0, 3->1, 4->4, 1->2, 0->2, 4->3, 3->0
# ---------------------------------------------------------------------------
SRC = np.array([0, 2, 1, 3, 4, 1, 0, 4, 3], np.uint32)
DST = np.array([1, 1, 0, 1, 4, 2, 2, 3, 0], np.uint32)
V5 = 5


def test_csc_known_answer():
    col, rows = orc.build_csc(V5, SRC, DST)
    # dst 0: [1, 3]; dst 1: [0, 2, 3]; dst 2: [1, 0]; dst 3: [4]; dst 4: [4]
    assert col.tolist() == [0, 2, 5, 7, 8, 9]
    assert rows.tolist() == [1, 3, 0, 2, 3, 1, 0, 4, 4]


def test_degrees_known_answer():
    out_d, in_d = orc.degrees(V5, SRC, DST)
    assert out_d.tolist() == [2, 2, 1, 2, 2]
    assert in_d.tolist() == [2, 3, 2, 1, 1]
    # clamp >= 1 (core/graph.hpp:4525-4530)
    out_d, in_d = orc.degrees(7, SRC, DST)
    assert out_d[5] == 1 and in_d[6] == 1


def test_sampler_full_neighbourhood_known_answer():
    col, rows = orc.build_csc(V5, SRC, DST)
    out_d, in_d = orc.degrees(V5, SRC, DST)
    s = orc.Sampler(col, rows, in_d, out_d, [5, 5])
    l0, l1 = s.sample(np.array([1, 3], np.uint32))
    # fanout >= degree -> all neighbours in CSC order, no draws
    assert l0["column_offset"].tolist() == [0, 3, 4]
    assert l0["sample_ans"].tolist() == [0, 2, 3, 4]
    assert l0["source"].tolist() == [0, 2, 3, 4]          # ascending
    assert l0["row_indices"].tolist() == [0, 1, 2, 3]
    # CSR: per src ascending dst
    assert l0["row_offset"].tolist() == [0, 1, 2, 3, 4]
    assert l0["column_indices"].tolist() == [0, 0, 0, 1]
    # weights 1/(sqrt(out[src]) * sqrt(in[dst])) in float32
    w = [np.float32(1) / (np.float32(np.sqrt(out_d[a])) * np.float32(np.sqrt(in_d[b])))
         for a, b in [(0, 1), (2, 1), (3, 1), (4, 3)]]
    np.testing.assert_array_equal(l0["edge_weight_forward"], np.array(w, np.float32))
    # layer 1 destinations = layer 0 source
    assert l1["destination"].tolist() == [0, 2, 3, 4]
    assert l1["sample_ans"].tolist() == [1, 3, 1, 0, 4, 4]
    assert l1["source"].tolist() == [0, 1, 3, 4]


def test_fuse_fwd_all_ones_is_weight_row_sum():
    col, rows = orc.build_csc(V5, SRC, DST)
    out_d, in_d = orc.degrees(V5, SRC, DST)
    s = orc.Sampler(col, rows, in_d, out_d, [5])
    (l0,) = s.sample(np.array([0, 1, 2], np.uint32))
    X = np.ones((l0["src_size"], 7), np.float32)
    Y = orc.fuse_fwd(l0, X, out_d, in_d)
    co, wf = l0["column_offset"], l0["edge_weight_forward"]
    for d in range(3):
        acc = np.float32(0)
        for e in range(co[d], co[d + 1]):
            acc = np.float32(acc + wf[e])
        assert np.all(Y[d] == acc)


# ---------------------------------------------------------------------------
# Cora (the reference's own data files)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def cora(golden):
    src, dst = dataloader.read_edge_file(golden / "cora" / "cora.2708.edge.self")
    V = 2708
    col, rows = orc.build_csc(V, src, dst)
    out_d, in_d = orc.degrees(V, src, dst)
    return dict(V=V, src=src, dst=dst, col=col, rows=rows, out_d=out_d, in_d=in_d)


def test_cora_files_parse(golden):
    src, dst = dataloader.read_edge_file(golden / "cora" / "cora.2708.edge.self")
    assert src.size == 13566 and int(max(src.max(), dst.max())) == 2707
    F, Lb, M = dataloader.read_feature_label_mask(
        golden / "cora" / "cora.featuretable.zip", golden / "cora" / "cora.labeltable",
        golden / "cora" / "cora.mask", 2708, 1433)
    assert F.shape == (2708, 1433) and set(np.unique(F)) <= {0.0, 1.0}
    assert Lb.min() == 0 and Lb.max() == 6
    assert int((M == 0).sum()) == 1605  # 1,605 train seeds


def test_cora_csc_matches_stable_sort(cora):
    order = np.argsort(cora["dst"], kind="stable")
    assert np.array_equal(cora["rows"], cora["src"][order])
    cnt = np.bincount(cora["dst"], minlength=cora["V"])
    assert np.array_equal(np.diff(cora["col"].astype(np.int64)), cnt)


def _python_reference_layer(dsts, col, rows, fanout, words):
    """Independent restatement of sample_processing1's draws: raw mt19937
    words (numpy MT19937, legacy seeding == std::mt19937(seed)), Lemire
    uniform_int_distribution, insert-until-size==num."""
    sets = []
    it = iter(words)
    for d in dsts:
        beg, end = int(col[d]), int(col[d + 1])
        deg = end - beg
        num = deg if fanout < 0 else min(deg, fanout)
        if fanout >= 0 and deg > fanout:
            thr = ((1 << 32) - deg) % deg
            chosen = set()
            while len(chosen) < num:
                while True:
                    m = int(next(it)) * deg
                    if (m & 0xFFFFFFFF) >= thr:
                        break
                chosen.add(m >> 32)
            sets.append(sorted(int(rows[beg + p]) for p in chosen))
        else:
            sets.append(sorted(int(x) for x in rows[beg:end]))
    return sets


def test_cora_mt19937_draws_match_independent_restatement(cora):
    rs = np.random.default_rng(5)
    seeds = rs.choice(cora["V"], 64, replace=False).astype(np.uint32)
    s = orc.Sampler(cora["col"], cora["rows"], cora["in_d"], cora["out_d"], [3, 2], seed=2000,
                    rng_mode=orc.RNG_MT_LEMIRE, order_mode=orc.ORDER_UNORDERED_MAP)
    l0, l1 = s.sample(seeds)
    bg = np.random.MT19937(0)
    bg._legacy_seeding(2000)
    words = bg.random_raw(200000)
    it = iter(words)

    class _Words:  # shared iterator across layers (one thread_local generator)
        def __iter__(self):
            return it

    for layer, fan in ((l0, 3), (l1, 2)):
        expect = _python_reference_layer(layer["destination"], cora["col"], cora["rows"], fan, _Words())
        co = layer["column_offset"]
        got = [sorted(layer["sample_ans"][co[k]:co[k + 1]].tolist()) for k in range(layer["v_size"])]
        assert got == expect


def test_cora_sampler_invariants_and_determinism(cora):
    seeds = np.arange(0, 2708, 37, dtype=np.uint32)
    runs = []
    for _ in range(2):
        s = orc.Sampler(cora["col"], cora["rows"], cora["in_d"], cora["out_d"], [25, 10])
        runs.append(s.sample(seeds))
    for a, b in zip(*runs):
        for k in ("column_offset", "sample_ans", "source", "row_indices", "row_offset",
                  "column_indices", "edge_weight_forward"):
            assert np.array_equal(a[k], b[k]), k
    col, rows = cora["col"], cora["rows"]
    for lay, fan in zip(runs[0], (25, 10)):
        co, ans = lay["column_offset"], lay["sample_ans"]
        assert np.all(np.diff(lay["source"].astype(np.int64)) > 0)
        assert np.all(lay["row_indices"] < lay["src_size"])
        assert np.array_equal(lay["source"][lay["row_indices"]], ans)
        for k, d in enumerate(lay["destination"]):
            nb = rows[col[d]:col[d + 1]]
            got = ans[co[k]:co[k + 1]]
            assert got.size == min(nb.size, fan)
            assert np.isin(got, nb).all()
            # distinct positions: every id at most as often as it occurs in the
            # neighbour list (cora.2708.edge.self contains duplicate edges)
            ids, cnt = np.unique(got, return_counts=True)
            avail = {int(a): int(c) for a, c in zip(*np.unique(nb, return_counts=True))}
            assert all(c <= avail[int(i)] for i, c in zip(ids, cnt))


def test_fuse_fwd_matches_numpy_float32(cora):
    s = orc.Sampler(cora["col"], cora["rows"], cora["in_d"], cora["out_d"], [25, 10])
    l0, l1 = s.sample(np.arange(0, 2708, 53, dtype=np.uint32))
    rng = np.random.default_rng(0)
    X = rng.standard_normal((l1["src_size"], 33)).astype(np.float32)
    Y = orc.fuse_fwd(l1, X, cora["out_d"], cora["in_d"])
    co, ri, wf = l1["column_offset"], l1["row_indices"], l1["edge_weight_forward"]
    ref = np.zeros_like(Y)
    for d in range(l1["v_size"]):
        acc = np.zeros(33, np.float32)
        for e in range(co[d], co[d + 1]):
            acc = (X[ri[e]] * wf[e]).astype(np.float32) + acc
        ref[d] = acc
    np.testing.assert_array_equal(Y, ref)
    # backward (deterministic restatement) == CSR gather in CSR order
    G = rng.standard_normal((l1["v_size"], 33)).astype(np.float32)
    Gin = orc.fuse_bwd(l1, G, cora["out_d"], cora["in_d"])
    ro, ci, wb = l1["row_offset"], l1["column_indices"], l1["edge_weight_backward"]
    ref = np.zeros_like(Gin)
    for r in range(l1["src_size"]):
        acc = np.zeros(33, np.float32)
        for j in range(ro[r], ro[r + 1]):
            acc = acc + (G[ci[j]] * wb[j]).astype(np.float32)
        ref[r] = acc
    np.testing.assert_array_equal(Gin, ref)


def test_cache_select_oracle_degree_order():
    """cache_high_degree + mark_cache_node restated (GS_SAMPLE_PD_CACHE.hpp:1019-1047):
    the cached set is the n highest out-degrees, slots follow (degree desc, id asc),
    and the two-tier gather returns exactly get_feature's rows."""
    rng = np.random.default_rng(5)
    deg = rng.integers(1, 20, 500).astype(np.uint32)
    for n in (0, 1, 37, 500):
        cmap, ids = orc.cache_select(deg, n)
        assert ids.size == n and np.array_equal(cmap[ids], np.arange(n, dtype=np.uint32))
        assert (cmap != orc.NOT_CACHED).sum() == n
        if 0 < n < 500:
            hot = deg[ids]
            assert hot.min() >= deg[cmap == orc.NOT_CACHED].max()
            assert all(hot[i] > hot[i + 1] or ids[i] < ids[i + 1] for i in range(n - 1))
        table = rng.standard_normal((500, 9)).astype(np.float32)
        idx = rng.integers(0, 500, 300).astype(np.uint32)
        cache = table[ids] if n else np.zeros((0, 9), np.float32)
        assert np.array_equal(orc.get_feature_cached(idx, cache, cmap, table), table[idx])


def _ogb_edges_loop(src, dst, n):
    """Line-by-line restatement of transOGBData_To_NeutronStarData.py's edge steps."""
    rows = list(zip(src.tolist(), dst.tolist())) + [(i, i) for i in range(n)]
    rows = sorted(rows, key=lambda r: r[0])  # (stable here; pandas quicksort is not)
    out = []
    for a, b in rows:
        out.append((b, a))
        out.append((a, b))
    seen, res = set(), []
    for p in out:
        if p not in seen:
            seen.add(p)
            res.append(p)
    return res


def test_ogb_edge_conversion_matches_loop_restatement():
    from nts import dataloader
    rng = np.random.default_rng(3)
    n = 50
    src = rng.integers(0, n, 300)
    dst = rng.integers(0, n, 300)
    s, d = dataloader.ogb_edges_to_reference(src, dst, n)
    assert list(zip(s.tolist(), d.tolist())) == _ogb_edges_loop(src, dst, n)
    pairs = set(zip(s.tolist(), d.tolist()))
    assert all((b, a) in pairs for a, b in pairs)  # symmetric
    assert all((i, i) in pairs for i in range(n))  # self-loops
    assert len(pairs) == s.size  # no duplicates


def test_convert_ogb_layout(tmp_path):
    from nts import dataloader
    root = tmp_path / "arxiv"
    for sub in ("raw/edge.csv", "raw/num-node-list.csv", "raw/node-label.csv", "raw/node-feat.csv",
                "split/time/train.csv", "split/time/valid.csv", "split/time/test.csv"):
        (root / sub).mkdir(parents=True)
    (root / "raw/num-node-list.csv/num-node-list.csv").write_text("5\n")
    (root / "raw/edge.csv/edge.csv").write_text("0,1\n3,2\n1,4\n")
    (root / "raw/node-label.csv/node-label.csv").write_text("\n".join("3 1 0 2 1".split()) + "\n")
    (root / "raw/node-feat.csv/node-feat.csv").write_text(
        "\n".join(f"{i}.5,{-i}.25" for i in range(5)) + "\n")
    (root / "split/time/train.csv/train.csv").write_text("4\n0\n")
    (root / "split/time/valid.csv/valid.csv").write_text("2\n")
    (root / "split/time/test.csv/test.csv").write_text("1\n3\n")
    p = dataloader.convert_ogb(root, "arxiv")
    s, d = dataloader.read_edge_file(p["edge"])
    assert list(zip(s.tolist(), d.tolist())) == _ogb_edges_loop(np.array([0, 3, 1]), np.array([1, 2, 4]), 5)
    feats, labels, masks = dataloader.read_feature_label_mask(p["feature"], p["label"], p["mask"], 5, 2)
    assert np.allclose(feats[:, 0], np.arange(5) + 0.5)
    assert np.allclose(feats[:, 1], [float(f"{-i}.25") for i in range(5)])
    assert labels.tolist() == [3, 1, 0, 2, 1]
    assert masks.tolist() == [dataloader.MASK_TRAIN, dataloader.MASK_TEST, dataloader.MASK_VAL,
                              dataloader.MASK_TEST, dataloader.MASK_TRAIN]


def test_up_degree_weights_use_sampled_layer_degrees():
    """UP_DEGREE (SampledSubgraph::update_degrees, core/FullyRepGraph.hpp:189-207):
    in = sampled edges of the dst, out = sampled edges of the src, then
    nts_norm_degree (float of double sqrt, 1 / (a * b)); Mean divides by in."""
    from nts import dataloader
    src, dst = dataloader.read_edge_file(GOLDEN / "cora" / "cora.2708.edge.self")
    V = 2708
    col, rows = orc.build_csc(V, src, dst)
    od, idg = orc.degrees(V, src, dst)
    seeds = np.arange(0, V, 17, dtype=np.uint32)
    for wt in (orc.W_SUM, orc.W_MEAN):
        o = orc.Sampler(col, rows, idg, od, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
        for ly in o.sample(seeds, 0, wt | orc.W_UP_DEGREE):
            co, ri = ly["column_offset"].astype(np.int64), ly["row_indices"]
            ind = np.diff(co)
            outd = np.bincount(ri, minlength=ly["src_size"])
            dl = np.repeat(np.arange(ind.size), ind)
            a = np.sqrt(outd[ri].astype(np.float64)).astype(np.float32)
            b = np.sqrt(ind[dl].astype(np.float64)).astype(np.float32)
            w = np.float32(1) / (a * b)
            if wt == orc.W_MEAN:
                w = w / ind[dl].astype(np.float32)
            assert np.array_equal(ly["edge_weight_forward"], w)


def test_mean_sampled_weights_divide_by_sampled_count():
    """W_MEAN_SAMPLED restates the reference GPU kernel get_mean_weight
    (cuda/ntsCUDATransferKernel.cuh:319-342): the Sum weight
    1/(sqrtf(out[src]) sqrtf(in[dst])) over full-graph degrees, divided by the
    dst's sampled edge count (edges_num = end - start)."""
    src, dst = dataloader.read_edge_file(GOLDEN / "cora" / "cora.2708.edge.self")
    V = 2708
    col, rows = orc.build_csc(V, src, dst)
    od, idg = orc.degrees(V, src, dst)
    seeds = np.arange(3, V, 13, dtype=np.uint32)
    o = orc.Sampler(col, rows, idg, od, [25, 10], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    for ly in o.sample(seeds, 0, orc.W_MEAN_SAMPLED):
        co = ly["column_offset"].astype(np.int64)
        cnt = np.diff(co)
        dl = np.repeat(np.arange(cnt.size), cnt)
        g_src = ly["source"][ly["row_indices"]]
        g_dst = ly["destination"][dl]
        # sqrtf of the (exactly representable) integer degree == float(double sqrt)
        a = np.sqrt(od[g_src].astype(np.float32))
        b = np.sqrt(idg[g_dst].astype(np.float32))
        w = (np.float32(1) / (a * b)) / cnt[dl].astype(np.float32)
        assert np.array_equal(ly["edge_weight_forward"], w)
