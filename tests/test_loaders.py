"""The reference's on-disk formats at scale, against the
format definitions (core/graph.hpp:1129-1186, core/ntsDataloador.hpp:999-1064,
core/ntsBaseOp.hpp:427-497) and the reference's own Cora files."""
import numpy as np
import pytest

from conftest import GOLDEN
from nts import dataloader


def test_edge_file_chunked_reads_round_trip(tmp_path):
    rng = np.random.default_rng(1)
    src = rng.integers(0, 2 ** 32, 100_003, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2 ** 32, 100_003, dtype=np.uint64).astype(np.uint32)
    p = tmp_path / "g.edge.bin"
    dataloader.write_edge_file(p, src, dst)
    assert p.stat().st_size == 8 * src.size
    assert dataloader.edge_count(p) == src.size
    s, d = dataloader.read_edges(p)
    assert np.array_equal(s, src) and np.array_equal(d, dst)
    for first, n in ((0, 1), (5, 1000), (99_000, 1003), (100_003, 0)):
        s, d = dataloader.read_edges(p, first, n)
        assert np.array_equal(s, src[first:first + n]) and np.array_equal(d, dst[first:first + n])
    with pytest.raises(IOError):
        dataloader.read_edges(p, 100_000, 10)
    (tmp_path / "bad.bin").write_bytes(b"\0" * 12)
    with pytest.raises(IOError):
        dataloader.edge_count(tmp_path / "bad.bin")


def test_cora_edges_match_the_raw_file():
    p = GOLDEN / "cora" / "cora.2708.edge.self"
    raw = np.fromfile(p, np.uint32).reshape(-1, 2)
    s, d = dataloader.read_edge_file(p)
    assert s.size == 13566 and np.array_equal(s, raw[:, 0]) and np.array_equal(d, raw[:, 1])


def test_native_text_reader_matches_numpy_restatement_on_cora():
    c = GOLDEN / "cora"
    a = dataloader.read_feature_label_mask(c / "cora.featuretable.zip", c / "cora.labeltable",
                                           c / "cora.mask", 2708, 1433)
    b = dataloader.read_feature_label_mask_numpy(c / "cora.featuretable.zip", c / "cora.labeltable",
                                                 c / "cora.mask", 2708, 1433)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)


def test_text_reader_lock_step_semantics(tmp_path):
    """Feature lines in any id order; the k-th label / mask lines belong to the
    k-th feature line whatever ids they carry; unlisted vertices keep their
    initial values; floats parse like istream (signs, exponents)."""
    (tmp_path / "f").write_text("3 1.5 -2e-3\n0 +4 5.25\n\n2 -0.0 7\n")
    (tmp_path / "l").write_text("99 6\n98 1\n97 2\n")
    (tmp_path / "m").write_text("9 test\n9 train\n9 val\n")
    f, l, m = dataloader.read_feature_label_mask(tmp_path / "f", tmp_path / "l", tmp_path / "m",
                                                 5, 2, threads=3)
    assert f[3].tolist() == [1.5, np.float32(-2e-3)] and f[0].tolist() == [4.0, 5.25]
    assert f[2].tolist() == [0.0, 7.0] and np.signbit(f[2, 0])
    assert l.tolist() == [1, 0, 2, 6, 0]
    assert m.tolist() == [dataloader.MASK_TRAIN, dataloader.MASK_UNLISTED, dataloader.MASK_VAL,
                          dataloader.MASK_TEST, dataloader.MASK_UNLISTED]
    (tmp_path / "f2").write_text("7 1 2\n")
    with pytest.raises(IOError):  # id past n_vertices
        dataloader.read_feature_label_mask(tmp_path / "f2", tmp_path / "l", tmp_path / "m", 5, 2)
    (tmp_path / "f3").write_text("1 1\n")
    with pytest.raises(IOError):  # fewer than F numbers
        dataloader.read_feature_label_mask(tmp_path / "f3", tmp_path / "l", tmp_path / "m", 5, 2)


def test_text_reader_files_smaller_than_the_thread_count(tmp_path):
    """Files of a few bytes cut for 16 threads: no cut may look before the text."""
    (tmp_path / "f").write_text("1 2\n")
    (tmp_path / "l").write_text("1 3\n")
    (tmp_path / "m").write_text("1 val\n")
    f, l, m = dataloader.read_feature_label_mask(tmp_path / "f", tmp_path / "l", tmp_path / "m",
                                                 2, 1, threads=16)
    assert f[1].tolist() == [2.0] and l.tolist() == [0, 3]
    assert m.tolist() == [dataloader.MASK_UNLISTED, dataloader.MASK_VAL]
    (tmp_path / "e").write_text("")
    f, l, m = dataloader.read_feature_label_mask(tmp_path / "e", tmp_path / "e", tmp_path / "e",
                                                 2, 1, threads=16)
    assert l.tolist() == [0, 0]


def test_text_reader_many_threads_large(tmp_path):
    rng = np.random.default_rng(3)
    V, F = 20_000, 16
    X = rng.standard_normal((V, F)).astype(np.float32)
    order = rng.permutation(V)
    lab = rng.integers(0, 40, V)
    with open(tmp_path / "f", "w") as fh:
        for v in order:
            fh.write(f"{v} " + " ".join(repr(float(x)) for x in X[v]) + "\n")
    with open(tmp_path / "l", "w") as fh:
        for v in order:
            fh.write(f"{v} {lab[v]}\n")
    with open(tmp_path / "m", "w") as fh:
        for v in order:
            fh.write(f"{v} {'train' if v % 3 == 0 else 'eval' if v % 3 == 1 else 'test'}\n")
    f, l, m = dataloader.read_feature_label_mask(tmp_path / "f", tmp_path / "l", tmp_path / "m",
                                                 V, F, threads=7)
    assert np.array_equal(f, X) and np.array_equal(l, lab)
    assert np.array_equal(m, np.arange(V) % 3)


def test_presample_file_round_trip_and_of_rate(tmp_path):
    counts = np.array([5, 0, 3, 7], np.uint32)
    ids = np.arange(15, dtype=np.uint32) * 11
    p = tmp_path / "x.pre_sample.bin"
    dataloader.write_presample_file(p, counts, ids)
    raw = np.fromfile(p, np.uint32)
    assert raw[:4].tolist() == counts.tolist() and np.array_equal(raw[4:], ids)
    k, got = dataloader.read_presample_file(p, 4)
    assert k.tolist() == counts.tolist() and np.array_equal(got, ids)
    # of_rate keeps the first (VertexId)(count * of_rate) ids of each super-batch
    k, got = dataloader.read_presample_file(p, 4, 0.5)
    assert k.tolist() == [2, 0, 1, 3]
    assert got.tolist() == [0, 11, 55, 88, 99, 110]
    assert dataloader.presample_file_name("./data/reddit.edge.self", 1024, "25-10", 4) == \
        "./data/reddit.edge.pre_sample_b1024_f25-10_p4.bin"


@pytest.mark.gpu
def test_edges_stream_to_device_in_chunks(tmp_path):
    import torch
    rng = np.random.default_rng(2)
    src = rng.integers(0, 2 ** 32, 50_001, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2 ** 32, 50_001, dtype=np.uint64).astype(np.uint32)
    p = tmp_path / "g.bin"
    dataloader.write_edge_file(p, src, dst)
    s, d = dataloader.load_edges_to_device(p, torch.device("cuda:0"), chunk=4096)
    assert np.array_equal(s.cpu().numpy().view(np.uint32), src)
    assert np.array_equal(d.cpu().numpy().view(np.uint32), dst)
