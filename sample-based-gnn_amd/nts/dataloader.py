"""Reference on-disk formats and the config parser.

* Edge file: raw binary array of {uint32 src; uint32 dst} (EdgeUnit<Empty>,
  core/graph.hpp:1139-1140), |E| = bytes / 8.
* Feature file: text, one line per vertex `id f_1 ... f_F`
  (GNNDatum::readFeature_Label_Mask, core/ntsDataloador.hpp:999-1064).
* Label file: `id label`; mask file: `id train|val|eval|test`; unlisted
  vertices keep the memset(…,1) pattern (core/ntsDataloador.hpp:191) = 0x01010101.
* FEATURE_FILE:random (core/ntsDataloador.hpp:835-861): all-ones features,
  rand() % C labels, masks 65/10/25 % by vertex id.
* Config: KEY:VALUE lines, `#` comments (InputInfo::readFromCfgFile,
  core/GraphSegment.cpp:222-347).
"""
from __future__ import annotations

import ctypes as C
import io
import os
import pathlib
import tempfile
import zipfile
from dataclasses import dataclass, field

import numpy as np

MASK_TRAIN, MASK_VAL, MASK_TEST, MASK_OTHER = 0, 1, 2, 3
MASK_UNLISTED = 0x01010101

_IO_PATH = pathlib.Path(__file__).resolve().parent / "lib" / "libnts_io.so"
_io_lib = None


def _io():
    """libnts_io.so (include/nts_io.h): the native loaders (built by build())."""
    global _io_lib
    if _io_lib is None:
        if not _IO_PATH.exists():
            raise ImportError(f"{_IO_PATH} missing: run __graft_entry__.build()")
        L = C.CDLL(str(_IO_PATH))
        L.nts_io_last_error.restype = C.c_char_p
        L.nts_io_edge_count.argtypes = [C.c_char_p]
        L.nts_io_edge_count.restype = C.c_int64
        L.nts_io_read_edges.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p]
        L.nts_io_read_feature_label_mask.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p,
                                                     C.c_uint64, C.c_uint32, C.c_void_p,
                                                     C.c_void_p, C.c_void_p, C.c_int]
        _io_lib = L
    return _io_lib


def _io_check(rc):
    if rc != 0:
        raise IOError(_io().nts_io_last_error().decode(errors="replace"))


def edge_count(path) -> int:
    n = _io().nts_io_edge_count(str(path).encode())
    if n < 0:
        raise IOError(_io().nts_io_last_error().decode(errors="replace"))
    return int(n)


def read_edges(path, first: int = 0, count: int | None = None):
    """Edges [first, first + count) of a binary edge file (memory-mapped read)."""
    E = edge_count(path)
    count = E - first if count is None else count
    src = np.empty(count, np.uint32)
    dst = np.empty(count, np.uint32)
    _io_check(_io().nts_io_read_edges(str(path).encode(), first, count,
                                      src.ctypes.data_as(C.c_void_p), dst.ctypes.data_as(C.c_void_p)))
    return src, dst


def read_edge_file(path) -> tuple[np.ndarray, np.ndarray]:
    return read_edges(path)


def load_edges_to_device(path, device, chunk: int = 1 << 26):
    """Stream a binary edge file of any size into int32 device tensors
    (src, dst) in chunks of `chunk` edges through a pinned staging buffer:
    host memory stays bounded by the chunk, not the file (FullyRepGraph then
    builds the CSC on the device, nts_hip_build_csc)."""
    import torch
    E = edge_count(path)
    src = torch.empty(E, dtype=torch.int32, device=device)
    dst = torch.empty(E, dtype=torch.int32, device=device)
    stage = [torch.empty((2, min(chunk, max(E, 1))), dtype=torch.int32).pin_memory() for _ in range(2)]
    ev = [None, None]
    for i, first in enumerate(range(0, E, chunk)):
        n = min(chunk, E - first)
        buf = stage[i % 2]
        if ev[i % 2] is not None:
            ev[i % 2].synchronize()  # the previous copy out of this buffer is done
        a = buf[0, :n].numpy().view(np.uint32)
        b = buf[1, :n].numpy().view(np.uint32)
        _io_check(_io().nts_io_read_edges(str(path).encode(), first, n,
                                          a.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p)))
        src[first:first + n].copy_(buf[0, :n], non_blocking=True)
        dst[first:first + n].copy_(buf[1, :n], non_blocking=True)
        ev[i % 2] = torch.cuda.Event()
        ev[i % 2].record()
    torch.cuda.synchronize(device)
    return src, dst


def write_edge_file(path, src: np.ndarray, dst: np.ndarray) -> None:
    e = np.empty((src.size, 2), np.uint32)
    e[:, 0] = src
    e[:, 1] = dst
    e.tofile(path)


def _text(path) -> str:
    p = pathlib.Path(path)
    if p.suffix == ".zip":
        with zipfile.ZipFile(p) as z:
            name = z.namelist()[0]
            return z.read(name).decode()
    return p.read_text()


def _plain_file(path, tmpdir):
    """The path itself, or the member of a one-file .zip extracted to tmpdir
    (the reference ships cora.featuretable zipped)."""
    p = pathlib.Path(path)
    if p.suffix != ".zip":
        return p
    with zipfile.ZipFile(p) as z:
        name = z.namelist()[0]
        out = pathlib.Path(tmpdir) / pathlib.Path(name).name
        out.write_bytes(z.read(name))
    return out


def read_feature_label_mask(feature_path, label_path, mask_path, n_vertices: int, n_features: int,
                            threads: int | None = None):
    """readFeature_Label_Mask (core/ntsDataloador.hpp:999-1064) for one partition
    covering all ids, parsed natively in parallel (libnts_io.so): the k-th
    feature, label and mask lines belong together, the vertex id is the feature
    line's; unlisted vertices keep zero features / label 0 / mask 0x01010101."""
    feats = np.zeros((n_vertices, n_features), np.float32)
    labels = np.zeros(n_vertices, np.int64)
    masks = np.full(n_vertices, MASK_UNLISTED, np.int32)
    threads = threads or min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS") or 16))
    with tempfile.TemporaryDirectory() as td:
        fp, lp, mp = (_plain_file(x, td) for x in (feature_path, label_path, mask_path))
        _io_check(_io().nts_io_read_feature_label_mask(
            str(fp).encode(), str(lp).encode(), str(mp).encode(), n_vertices, n_features,
            feats.ctypes.data_as(C.c_void_p), labels.ctypes.data_as(C.c_void_p),
            masks.ctypes.data_as(C.c_void_p), threads))
    return feats, labels, masks


def read_feature_label_mask_numpy(feature_path, label_path, mask_path, n_vertices: int,
                                  n_features: int):
    """A plain numpy restatement of the same reader (small files; tests)."""
    feats = np.zeros((n_vertices, n_features), np.float32)
    labels = np.zeros(n_vertices, np.int64)
    masks = np.full(n_vertices, MASK_UNLISTED, np.int32)
    ftab = np.loadtxt(io.StringIO(_text(feature_path)), dtype=np.float64, ndmin=2)
    ids = ftab[:, 0].astype(np.int64)
    feats[ids] = ftab[:, 1:1 + n_features].astype(np.float32)
    ltab = np.loadtxt(io.StringIO(_text(label_path)), dtype=np.int64, ndmin=2)
    labels[ids] = ltab[: ids.size, 1]
    kinds = {"train": MASK_TRAIN, "eval": MASK_VAL, "val": MASK_VAL, "test": MASK_TEST}
    mlines = _text(mask_path).split()
    mvals = np.array([kinds.get(s, MASK_OTHER) for s in mlines[1::2]], np.int32)
    masks[ids] = mvals[: ids.size]
    return feats, labels, masks


# ---------------------------------------------------------------------------
# PRE_SAMPLE_FILE (core/ntsBaseOp.hpp:427-497): the hot vertices of every
# super-batch found by preSample, as
#   uint32 counts[S]            (vertices of super-batch 0 .. S-1)
#   uint32 ids[sum(counts)]     (super-batch 0's ids, then 1's, ...)
# ---------------------------------------------------------------------------
def presample_file_name(edge_file, batch_size: int, fanout_string: str, pipeline_num: int) -> str:
    """Default name when PRE_SAMPLE_FILE is unset or missing (:432-439):
    <edge file up to its last '.'>.pre_sample_b<B>_f<fanout>_p<pipeline>.bin"""
    e = str(edge_file)
    dot = e.rfind(".")
    return e[:dot + 1] + f"pre_sample_b{batch_size}_f{fanout_string}_p{pipeline_num}.bin"


def write_presample_file(path, counts, ids) -> None:
    counts = np.ascontiguousarray(counts, np.uint32)
    ids = np.ascontiguousarray(ids, np.uint32)
    if int(counts.sum(dtype=np.uint64)) != ids.size:
        raise ValueError("ids must hold sum(counts) vertices")
    with open(path, "wb") as f:
        f.write(counts.tobytes())
        f.write(ids.tobytes())


def read_presample_file(path, n_super_batches: int, of_rate: float = 1.0):
    """The reader of :475-497: per super-batch i keep its first
    (VertexId)(counts[i] * of_rate) ids.  Returns (kept counts, concatenated ids)."""
    raw = np.fromfile(path, dtype=np.uint32)
    if raw.size < n_super_batches:
        raise ValueError(f"{path}: fewer than {n_super_batches} counts")
    counts = raw[:n_super_batches].astype(np.uint64)
    body = raw[n_super_batches:]
    if int(counts.sum()) > body.size:
        raise ValueError(f"{path}: truncated id section")
    keep = np.array([int(np.float32(c) * np.float32(of_rate)) for c in counts], np.uint32)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    ids = np.concatenate([body[s:s + k] for s, k in zip(starts, keep)]) if keep.size else body[:0]
    return keep, ids.astype(np.uint32)


def random_generate(n_vertices: int, n_features: int, n_classes: int, seed: int = 1,
                    train_rate=0.65, val_rate=0.10):
    """GNNDatum::random_generate: all-ones features, uniform labels, masks by id."""
    feats = np.ones((n_vertices, n_features), np.float32)
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, n_classes, n_vertices).astype(np.int64)
    max_train = int(n_vertices * train_rate)
    max_val = int(n_vertices * val_rate + max_train)
    masks = np.full(n_vertices, MASK_TEST, np.int32)
    masks[:max_train] = MASK_TRAIN
    masks[max_train:max_val] = MASK_VAL
    return feats, labels, masks


@dataclass
class InputInfo:
    """InputInfo (core/GraphSegment.h:156-244) — the cfg keys of Appendix C."""
    algorithm: str = ""
    vertices: int = 0
    epochs: int = 0
    layer_string: str = ""
    fanout_string: str = ""
    edge_file: str = ""
    feature_file: str = ""
    label_file: str = ""
    mask_file: str = ""
    learn_rate: float = 0.0
    weight_decay: float = 0.0
    decay_rate: float = 0.0
    decay_epoch: float = 0.0
    drop_rate: float = 0.0
    batch_size: int = 0
    pipeline_num: int = 1
    cache_rate: float = 0.1
    up_degree: bool = False
    gpu_num: int = 1
    pre_sample_file: str = ""
    extra: dict = field(default_factory=dict)

    @property
    def layers(self) -> list[int]:
        return [int(x) for x in self.layer_string.split("-") if x]

    @property
    def fanout(self) -> list[int]:
        return [int(x) for x in self.fanout_string.split("-") if x]

    @classmethod
    def from_cfg(cls, path) -> "InputInfo":
        info = cls()
        keymap = {
            "ALGORITHM": ("algorithm", str), "VERTICES": ("vertices", int), "EPOCHS": ("epochs", int),
            "LAYERS": ("layer_string", str), "FANOUT": ("fanout_string", str),
            "EDGE_FILE": ("edge_file", str), "FEATURE_FILE": ("feature_file", str),
            "LABEL_FILE": ("label_file", str), "MASK_FILE": ("mask_file", str),
            "LEARN_RATE": ("learn_rate", float), "WEIGHT_DECAY": ("weight_decay", float),
            "DECAY_RATE": ("decay_rate", float), "DECAY_EPOCH": ("decay_epoch", float),
            "DROP_RATE": ("drop_rate", float), "BATCH_SIZE": ("batch_size", int),
            "PIPELINE_NUM": ("pipeline_num", int), "CACHE_RATE": ("cache_rate", float),
            "UP_DEGREE": ("up_degree", lambda s: bool(int(s))), "GPU_NUM": ("gpu_num", int),
            "PRE_SAMPLE_FILE": ("pre_sample_file", str),
        }
        for raw in pathlib.Path(path).read_text().splitlines():
            line = raw.strip()
            if not line or line.startswith("#") or ":" not in line:
                continue
            k, v = line.split(":", 1)
            k, v = k.strip(), v.strip()
            if k in keymap:
                name, conv = keymap[k]
                setattr(info, name, conv(v))
            else:
                info.extra[k] = v
        return info


# ---------------------------------------------------------------------------
# OGB node-property datasets -> the reference's on-disk formats
# ---------------------------------------------------------------------------
OGB_SPLIT = {"products": "sales_ranking", "proteins": "species", "proteinfunc": "species"}


def ogb_edges_to_reference(src: np.ndarray, dst: np.ndarray, n_vertices: int):
    """Edge list of transOGBData_To_NeutronStarData.py (data/OGBData/, lines 17-50):
    append a self-loop per vertex, sort by source, emit (dst, src) then (src, dst)
    for every row, drop repeated pairs keeping the first occurrence.  The
    reference sorts with pandas' default (unstable) quicksort; equal sources
    keep their file order here."""
    a = np.concatenate([np.asarray(src, np.int64), np.arange(n_vertices, dtype=np.int64)])
    b = np.concatenate([np.asarray(dst, np.int64), np.arange(n_vertices, dtype=np.int64)])
    order = np.argsort(a, kind="stable")
    a, b = a[order], b[order]
    s = np.empty(2 * a.size, np.int64)
    d = np.empty(2 * a.size, np.int64)
    s[0::2], d[0::2] = b, a  # reverse edge first (":my_output_file.write(row[1], row[0])")
    s[1::2], d[1::2] = a, b
    key = s * np.int64(n_vertices) + d
    _, first = np.unique(key, return_index=True)
    keep = np.sort(first)
    return s[keep].astype(np.uint32), d[keep].astype(np.uint32)


def convert_ogb(root, name: str, out_dir=None) -> dict:
    """Convert an OGB node-property dataset laid out as the reference expects
    (`<root>/raw/edge.csv/edge.csv`, `raw/num-node-list.csv/...`,
    `raw/node-label.csv/...`, `raw/node-feat.csv/...`,
    `split/<split>/{train,valid,test}.csv/...`) into the reference's files:
    `<name>.edge.self.bin` (binary u32 pairs, convert2binary.cpp),
    `<name>.featuretable` (`id f...`), `<name>.labeltable` (`id label`),
    `<name>.mask` (`id train|eval|test`, sorted by id).  Returns the paths."""
    root = pathlib.Path(root)
    out = pathlib.Path(out_dir) if out_dir else root / "Data"
    out.mkdir(parents=True, exist_ok=True)
    raw = root / "raw"
    n = int(np.loadtxt(raw / "num-node-list.csv" / "num-node-list.csv", delimiter=",", ndmin=1)[0])
    e = np.loadtxt(raw / "edge.csv" / "edge.csv", delimiter=",", dtype=np.int64, ndmin=2)
    s, d = ogb_edges_to_reference(e[:, 0], e[:, 1], n)
    paths = {"edge": out / f"{name}.edge.self.bin", "feature": out / f"{name}.featuretable",
             "label": out / f"{name}.labeltable", "mask": out / f"{name}.mask"}
    write_edge_file(paths["edge"], s, d)
    labels = np.loadtxt(raw / "node-label.csv" / "node-label.csv", delimiter=",", dtype=str, ndmin=2)
    with open(paths["label"], "w") as f:
        for i, row in enumerate(labels):
            f.write(f"{i} {' '.join(row)}\n")
    feats = np.loadtxt(raw / "node-feat.csv" / "node-feat.csv", delimiter=",", dtype=str, ndmin=2)
    with open(paths["feature"], "w") as f:
        for i, row in enumerate(feats):
            f.write(f"{i} {' '.join(row)}\n")
    split = root / "split" / OGB_SPLIT.get(name, "time")
    ids, kinds = [], []
    for part, tag in (("train", "train"), ("valid", "eval"), ("test", "test")):
        v = np.loadtxt(split / f"{part}.csv" / f"{part}.csv", delimiter=",", dtype=np.int64, ndmin=1)
        ids.append(v.reshape(-1))
        kinds += [tag] * v.size
    ids = np.concatenate(ids)
    order = np.argsort(ids, kind="stable")
    with open(paths["mask"], "w") as f:
        for k in order:
            f.write(f"{ids[k]} {kinds[k]}\n")
    return paths
