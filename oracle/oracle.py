"""ORACLE — test infrastructure only (see ref_cpu.cpp header).

numpy/ctypes wrappers over oracle/build/liboracle.so, a CPU restatement of the
reference's GCN_CPU_SAMPLE hot path.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product never does.
"""
from __future__ import annotations

import ctypes as C
import pathlib
import subprocess

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
LIB = HERE / "build" / "liboracle.so"
# build variants: "O3" (-O3 x86-64-v3, the checker and the CPU baseline) and
# "O0" (the reference's shipped -O0 flags, a secondary baseline figure)
LIBS = {"O3": LIB, "O0": HERE / "build" / "liboracle_O0.so"}

RNG_PHILOX, RNG_MT_LEMIRE, RNG_MT_DIV = 0, 1, 2
ORDER_DRAW, ORDER_UNORDERED_MAP = 0, 1
W_SUM, W_MEAN, W_NONE, W_MEAN_SAMPLED = 0, 1, 2, 3
W_UP_DEGREE = 0x10  # OR-ed into the weight type: UP_DEGREE per-layer degrees
F_MERGE_SRC_DST = 0x20  # OR-ed: dsts merged into the frontier (GAT), dst_local_id

_libs = {}
_active = "O3"


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


class variant:
    """`with oracle.variant("O0"):` — calls (and Samplers created) inside use
    that build of ref_cpu.cpp."""

    def __init__(self, name: str):
        if name not in LIBS:
            raise ValueError(name)
        self.name = name

    def __enter__(self):
        global _active
        self.prev, _active = _active, self.name
        return self

    def __exit__(self, *exc):
        global _active
        _active = self.prev


def lib():
    if _active not in _libs:
        path = LIBS[_active]
        if not path.exists():
            build()
        L = C.CDLL(str(path))
        P, U32, U64, I = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
        L.orc_build_csc.argtypes = [U64, U64, P, P, P, P]
        L.orc_degrees.argtypes = [U64, U64, P, P, P, P]
        L.orc_sampler_new.argtypes = [U64, P, P, P, P, I, P, U64, I, I]
        L.orc_sampler_new.restype = P
        L.orc_sampler_free.argtypes = [P]
        L.orc_sample_batch.argtypes = [P, P, U32, U64, I, I, I]
        L.orc_layer_size.argtypes = [P, I, P]
        L.orc_layer_copy.argtypes = [P, I] + [P] * 9
        L.orc_mt_state.argtypes = [P, P]
        L.orc_layer_extra.argtypes = [P, I, P, P]
        L.orc_get_feature.argtypes = [U32, P, P, U32, P, I]
        L.orc_fuse_fwd.argtypes = [U32, P, P, P, P, P, P, P, U32, P, I, I]
        L.orc_fuse_bwd.argtypes = [U32, U32, P, P, P, P, P, P, P, U32, P, I, I]
        L.orc_sampler_set_omit.argtypes = [P, P, U32]
        L.orc_pushdown_fwd.argtypes = [U32, U32, P, P, P, P, P, U32, P]
        L.orc_presample.argtypes = [U64, P, P, P, U32, I, C.c_float, P, P, P]
        _libs[_active] = L
    return _libs[_active]


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def build_csc(V: int, src: np.ndarray, dst: np.ndarray):
    src = np.ascontiguousarray(src, np.uint32)
    dst = np.ascontiguousarray(dst, np.uint32)
    col = np.empty(V + 1, np.uint64)
    rows = np.empty(src.size, np.uint32)
    lib().orc_build_csc(V, src.size, _p(src), _p(dst), _p(col), _p(rows))
    return col, rows


def degrees(V: int, src: np.ndarray, dst: np.ndarray):
    src = np.ascontiguousarray(src, np.uint32)
    dst = np.ascontiguousarray(dst, np.uint32)
    out_d = np.empty(V, np.uint32)
    in_d = np.empty(V, np.uint32)
    lib().orc_degrees(V, src.size, _p(src), _p(dst), _p(out_d), _p(in_d))
    return out_d, in_d


class Sampler:
    """FastSampler::sample_fast restated (single sampler thread unless threads > 1)."""

    def __init__(self, col, rows, in_deg, out_deg, fanout, seed=2000, rng_mode=RNG_MT_LEMIRE,
                 order_mode=ORDER_UNORDERED_MAP):
        self.col = np.ascontiguousarray(col, np.uint64)
        self.rows = np.ascontiguousarray(rows, np.uint32)
        self.in_deg = np.ascontiguousarray(in_deg, np.uint32)
        self.out_deg = np.ascontiguousarray(out_deg, np.uint32)
        self.fanout = np.ascontiguousarray(fanout, np.int32)
        self.L = len(fanout)
        V = self.col.size - 1
        self.L_ = lib()
        self.h = self.L_.orc_sampler_new(V, _p(self.col), _p(self.rows), _p(self.in_deg),
                                       _p(self.out_deg), self.L, _p(self.fanout), seed, rng_mode,
                                       order_mode)

    def __del__(self):
        if getattr(self, "h", None):
            self.L_.orc_sampler_free(self.h)
            self.h = None

    def set_omit(self, omit_map=None, omit_key=0):
        """sample_gpu_fast_omit: in the last layer, dsts with omit_map[d] == key
        sample nothing (None: off)."""
        self._omit = None if omit_map is None else np.ascontiguousarray(omit_map, np.uint32)
        self.L_.orc_sampler_set_omit(self.h, _p(self._omit), int(omit_key))

    def sample(self, seeds, batch_seq=0, weight_type=W_SUM, build_csr=True, threads=1):
        seeds = np.ascontiguousarray(seeds, np.uint32)
        self.L_.orc_sample_batch(self.h, _p(seeds), seeds.size, batch_seq, weight_type,
                               int(build_csr), threads)
        return [self.layer(l) for l in range(self.L)]

    def layer(self, l):
        sz = np.empty(3, np.uint32)
        self.L_.orc_layer_size(self.h, l, _p(sz))
        v, e, s = (int(x) for x in sz)
        out = dict(
            destination=np.empty(v, np.uint32), column_offset=np.empty(v + 1, np.uint32),
            row_indices=np.empty(e, np.uint32), sample_ans=np.empty(e, np.uint32),
            source=np.empty(s, np.uint32), edge_weight_forward=np.zeros(e, np.float32),
            row_offset=np.zeros(s + 1, np.uint32), column_indices=np.zeros(e, np.uint32),
            edge_weight_backward=np.zeros(e, np.float32))
        self.L_.orc_layer_copy(self.h, l, *[_p(out[k]) for k in (
            "destination", "column_offset", "row_indices", "sample_ans", "source",
            "edge_weight_forward", "row_offset", "column_indices", "edge_weight_backward")])
        out.update(v_size=v, e_size=e, src_size=s)
        dl, ce = np.zeros(v, np.uint32), np.zeros(e, np.uint32)
        have = self.L_.orc_layer_extra(self.h, l, _p(dl), _p(ce))
        if have & 1:
            out["dst_local_id"] = dl
        if have & 2:
            out["csr_edge_id"] = ce
        return out

    def mt_state(self):
        st = np.empty(625, np.uint32)
        self.L_.orc_mt_state(self.h, _p(st))
        return st


def get_feature(idx, table, threads=1):
    idx = np.ascontiguousarray(idx, np.uint32)
    table = np.ascontiguousarray(table, np.float32)
    out = np.empty((idx.size, table.shape[1]), np.float32)
    lib().orc_get_feature(idx.size, _p(idx), _p(table), table.shape[1], _p(out), threads)
    return out


def fuse_fwd(layer, X, out_deg, in_deg, weight_mean=False, threads=1):
    """MiniBatchFuseOp::forward over one sampled layer."""
    X = np.ascontiguousarray(X, np.float32)
    v = layer["v_size"]
    Y = np.empty((v, X.shape[1]), np.float32)
    lib().orc_fuse_fwd(v, _p(layer["column_offset"]), _p(layer["row_indices"]), _p(layer["source"]),
                       _p(layer["destination"]), _p(np.ascontiguousarray(out_deg, np.uint32)),
                       _p(np.ascontiguousarray(in_deg, np.uint32)), _p(X), X.shape[1], _p(Y),
                       int(weight_mean), threads)
    return Y


def fuse_bwd(layer, G, out_deg, in_deg, weight_mean=False, threads=1):
    """MiniBatchFuseOp::backward over one sampled layer."""
    G = np.ascontiguousarray(G, np.float32)
    v, s = layer["v_size"], layer["src_size"]
    Gin = np.empty((s, G.shape[1]), np.float32)
    lib().orc_fuse_bwd(v, s, _p(layer["column_offset"]), _p(layer["row_indices"]),
                       _p(layer["source"]), _p(layer["destination"]),
                       _p(np.ascontiguousarray(out_deg, np.uint32)),
                       _p(np.ascontiguousarray(in_deg, np.uint32)), _p(G), G.shape[1], _p(Gin),
                       int(weight_mean), threads)
    return Gin


NOT_CACHED = 0xFFFFFFFF


def cache_select(out_deg, n_cache):
    """Degree-ordered feature-cache selection of GS_SAMPLE_PD_CACHE
    (cache_high_degree + mark_cache_node, toolkits/GS_SAMPLE_PD_CACHE.hpp:1019-1047):
    vertex ids sorted by out_degree_for_backward descending, the first n_cache
    get slots 0, 1, ... in that order, every other vertex is not cached (-1).
    The reference's std::sort leaves equal degrees in an unspecified order; the
    tie rule restated here (ascending id) is this build's."""
    out_deg = np.asarray(out_deg, np.uint32)
    order = np.argsort(-out_deg.astype(np.int64), kind="stable").astype(np.uint32)
    cmap = np.full(out_deg.size, NOT_CACHED, np.uint32)
    cmap[order[:n_cache]] = np.arange(n_cache, dtype=np.uint32)
    return cmap, order[:n_cache].copy()


def get_feature_cached(idx, cache, cache_map, host_table):
    """load_feature_gpu_cache (core/ntsFastSampler.hpp:263-317): rows of cached
    vertices from the device cache, the others from the pinned host table."""
    idx = np.asarray(idx, np.uint32)
    slots = cache_map[idx]
    out = np.empty((idx.size, host_table.shape[1]), np.float32)
    hot = slots != NOT_CACHED
    out[hot] = cache[slots[hot]]
    out[~hot] = host_table[idx[~hot]]
    return out


def pushdown_fwd(layer, X, v_begin=0, v_end=None):
    """PushDownBatchOp::forward over dst rows [v_begin, v_end) of a sampled
    layer (global feature table X, the layer's forward weights)."""
    X = np.ascontiguousarray(X, np.float32)
    v_end = layer["v_size"] if v_end is None else v_end
    Y = np.empty((v_end - v_begin, X.shape[1]), np.float32)
    lib().orc_pushdown_fwd(v_begin, v_end, _p(layer["column_offset"]), _p(layer["row_indices"]),
                           _p(layer["source"]), _p(layer["edge_weight_forward"]), _p(X),
                           X.shape[1], _p(Y))
    return Y


def presample(col, rows, seeds, layers, cache_rate):
    """get_most_neighbor of one super-batch: (counts [V], hot ids)."""
    col = np.ascontiguousarray(col, np.uint64)
    rows = np.ascontiguousarray(rows, np.uint32)
    seeds = np.ascontiguousarray(seeds, np.uint32)
    V = col.size - 1
    counts = np.empty(V, np.uint32)
    ids = np.empty(V, np.uint32)
    n = np.zeros(1, np.uint32)
    lib().orc_presample(V, _p(col), _p(rows), _p(seeds), seeds.size, layers, float(cache_rate),
                        _p(counts), _p(ids), _p(n))
    return counts, ids[:int(n[0])].copy()
