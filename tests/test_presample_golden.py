"""The reference's one held output on the PD-cache path: its own preSample
result `data/cora.2708.edge.pre_sample_b1024_f25-10_p1.bin` (copied as data
into tests/golden/cora/), written by nts::op::preSample
(/root/reference/core/ntsBaseOp.hpp:427-473) and read back by :475-543.

What it pins, and what it cannot:
  * FORMAT (pinned): uint32 counts[S] then the ids of every super-batch in
    order.  Here S = 64 (64 + 101 + 96 + 63 = 324 words), the ids are < V,
    distinct and ascending inside each super-batch (the single-thread
    collection order of get_most_neighbor, :376-390), and each count is
    (VertexId)(total_sample_num * 0.8) for an integer total (the rate the
    writer forces, :418-420).  nts.dataloader.read_presample_file reads it
    exactly as the reference reader does, including the reference's reading
    of a header of the CURRENT run's super-batch count.
  * CONTENT (cannot match): the file was not produced from the shipped Cora
    inputs.  64 super-batches of 1024 seeds need > 63 * 1024 train ids, the
    Cora mask has 1605; 61 of the 64 counts are 0, which get_most_neighbor
    cannot return for a non-empty slice of train ids; and no seed set on
    cora.2708.edge.self yields super-batch 0's hot set under 1-hop counting
    (test below: even the union of the in-neighbourhoods of every admissible
    seed misses some of its ids).  The hot-set selection itself is pinned by
    the restatement tests in test_pdcache.py, not by this file.
"""
import pathlib

import numpy as np

from nts import dataloader

GOLD = pathlib.Path(__file__).parent / "golden" / "cora"
FILE = GOLD / "cora.2708.edge.pre_sample_b1024_f25-10_p1.bin"
V = 2708


def _sets(counts, ids):
    out, o = [], 0
    for n in counts:
        out.append(ids[o:o + int(n)])
        o += int(n)
    return out


def test_presample_file_format_golden():
    raw = np.fromfile(FILE, np.uint32)
    assert raw.size == 324
    counts, ids = dataloader.read_presample_file(FILE, 64)
    assert counts[:3].tolist() == [101, 96, 63] and not counts[3:].any()
    assert ids.size == 260 and int(ids.max()) < V
    for s in _sets(counts, ids):
        assert np.all(np.diff(s.astype(np.int64)) > 0)  # distinct, ascending
    # (VertexId)(total_sample_num * cache_rate) with cache_rate forced to 0.8
    for n in counts[:3]:
        assert any(int(np.float32(t) * np.float32(0.8)) == n for t in range(1, V + 2))
    # of_rate keeps the first (VertexId)(count * of_rate) ids of each super-batch
    k, got = dataloader.read_presample_file(FILE, 64, 0.5)
    assert k[:3].tolist() == [50, 48, 31]
    full = _sets(counts, ids)
    assert np.array_equal(got, np.concatenate([full[0][:50], full[1][:48], full[2][:31]]))


def test_reference_reader_with_the_shipped_cfg_header_length():
    """gcn_cora_sample.cfg (BATCH_SIZE 64, PIPELINE_NUM 4) has ceil(1605 / 256)
    = 7 super-batches: the reference reader takes 7 counts and seeks the ids
    from word 7 (:505-536), i.e. inside the file's 64-word header — it would
    load zeros as hot vertices.  The dataloader reproduces that reading."""
    counts, ids = dataloader.read_presample_file(FILE, 7)
    assert counts.tolist() == [101, 96, 63, 0, 0, 0, 0]
    assert ids.size == 260 and not ids[:57].any()


def test_hot_sets_are_not_from_the_shipped_cora_inputs():
    from oracle import oracle as orc
    src, dst = dataloader.read_edge_file(GOLD / "cora.2708.edge.self")
    col, rows = orc.build_csc(V, src, dst)
    counts, ids = dataloader.read_presample_file(FILE, 64)
    s0 = _sets(counts, ids)[0]
    hot, top = set(s0.tolist()), int(s0.max())
    nbrs = [rows[col[v]:col[v + 1]] for v in range(V)]
    # a seed is admissible iff its in-neighbours up to the set's maximum id all
    # lie in the hot set (hot = the lowest-id vertices of count >= pivot)
    admissible = [v for v in range(V) if all(u > top or u in hot for u in nbrs[v].tolist())]
    reach = set()
    for v in admissible:
        reach.update(u for u in nbrs[v].tolist() if u <= top)
    assert len(hot - reach) > 0
    # and the Cora train slice of the cfg's 1024-seed super-batch gives a hot
    # set of another size altogether
    mask = {}
    for line in open(GOLD / "cora.mask"):
        i, t = line.split()
        mask[int(i)] = t
    train = np.array(sorted(i for i, t in mask.items() if t == "train"), np.uint32)
    assert train.size == 1605
    _, h = orc.presample(col, rows, train[:1024], 2, 0.8)
    assert h.size != s0.size
