"""ctypes binding of the C-ABI in include/nts_hip.h (libnts_hip.so).

This is the same boundary a reference-side maintainer would bind (see
INTEGRATION.md); the C++ host layer (nts/host/*.cpp) links the library
directly.  Loading fails loudly when the HIP library is missing — there is no
CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

import torch  # noqa: F401  (must be loaded first: its HIP runtime is the one we share)

_HERE = pathlib.Path(__file__).resolve().parent
# NTS_HIP_LIB: another build of the same ABI (A/B builds of a tuning knob)
LIB_PATH = pathlib.Path(os.environ["NTS_HIP_LIB"]) if os.environ.get("NTS_HIP_LIB") else _HERE / "lib" / "libnts_hip.so"

NTS_OK = 0
ABI_VERSION = 11  # NTS_HIP_ABI_VERSION of the header these ctypes structs mirror
NTS_RNG_PHILOX = 0
NTS_RNG_MT19937_LEMIRE = 1
NTS_RNG_MT19937_DIV = 2
NTS_GEMM_F32 = 0
NTS_GEMM_SPLIT3 = 1
NTS_GEMM_SPLIT3_ALL = 2  # the split kernels for every shape they take (kernel tests)
NTS_WEIGHT_SUM = 0
NTS_WEIGHT_MEAN = 1
NTS_WEIGHT_NONE = 2
NTS_WEIGHT_MEAN_SAMPLED = 3

# every symbol declared in include/nts_hip.h (checked by tests/test_abi.py)
EXPORTED = (
    "nts_hip_abi_version", "nts_hip_last_error", "nts_hip_ctx_create", "nts_hip_ctx_destroy",
    "nts_hip_ctx_set_stream", "nts_hip_ctx_get_stream", "nts_hip_ctx_reserve",
    "nts_hip_ctx_set_gemm_mode", "nts_hip_ctx_get_gemm_mode",
    "nts_hip_rng_seed", "nts_hip_rng_state", "nts_hip_degrees", "nts_hip_build_csc",
    "nts_hip_sample_layer", "nts_hip_gather_rows", "nts_hip_gather_labels",
    "nts_hip_spmm_csc_fwd", "nts_hip_spmm_csr_bwd", "nts_hip_spmm_csc_bwd_atomic",
    "nts_hip_spmm_csc_fwd_act", "nts_hip_spmm_csr_bwd_masked", "nts_hip_gemm_gather_f32",
    "nts_hip_gemm_tn_gather_f32", "nts_hip_act_backward", "nts_hip_presample_counts",
    "nts_hip_presample_select", "nts_hip_pd_set_cache", "nts_hip_pd_load_share",
    "nts_hip_relu_dropout_f32",
    "nts_hip_gemm_f32", "nts_hip_gemm_relu_dropout_f32", "nts_hip_gemm_tn_masked_f32",
    "nts_hip_linear_xent_fwd", "nts_hip_linear_xent_bwd", "nts_hip_linear_xent_train", "nts_hip_adam", "nts_hip_comm_unique_id", "nts_hip_comm_init", "nts_hip_comm_destroy",
    "nts_hip_comm_count",
    "nts_hip_allreduce_sum_f32", "nts_hip_broadcast_f32",
    "nts_hip_cache_select", "nts_hip_host_alloc", "nts_hip_host_free",
    "nts_hip_host_device_pointer", "nts_hip_gather_rows_cached", "nts_hip_spmm_csc_fwd_cached",
    "nts_hip_stage_uncached_rows", "nts_hip_gat_forward", "nts_hip_gat_backward",
    "nts_hip_h2_split_rows", "nts_hip_gemm_h2_gather", "nts_hip_gemm_h2_tn_gather",
    "nts_hip_h2_split_rows_planar", "nts_hip_gemm_h2p_tn_gather", "nts_hip_gemm_h2p_gather",
    "nts_hip_spmm_csr_bwd_postmask", "nts_hip_spmm_csr_bwd_colmax", "nts_hip_gemm_h2p_tn_gather_cm",
    "nts_hip_csr_bwd_colmax_rows_per_part", "nts_hip_gemm_h2d_act",
    "nts_hip_act_bits_words", "nts_hip_spmm_csc_fwd_act_bits", "nts_hip_spmm_csr_bwd_postmask_bits",
    "nts_hip_mt_budget_scale", "nts_hip_mt_checkpoint", "nts_hip_mt_rewind",
)
NTS_NOT_CACHED = 0xFFFFFFFF


class GraphDev(C.Structure):
    """nts_graph_dev"""
    _fields_ = [
        ("n_vertices", C.c_uint64), ("n_edges", C.c_uint64),
        ("column_offset", C.c_void_p), ("row_indices", C.c_void_p),
        ("in_degree", C.c_void_p), ("out_degree", C.c_void_p),
    ]


class SampCSCDev(C.Structure):
    """nts_sampcsc_dev"""
    _fields_ = [
        ("v_cap", C.c_uint32), ("e_cap", C.c_uint32), ("s_cap", C.c_uint32),
        ("destination", C.c_void_p), ("v_size", C.c_void_p),
        ("column_offset", C.c_void_p), ("row_indices", C.c_void_p),
        ("sample_ans", C.c_void_p), ("edge_dst", C.c_void_p), ("source", C.c_void_p),
        ("edge_weight_forward", C.c_void_p), ("row_offset", C.c_void_p),
        ("column_indices", C.c_void_p), ("edge_weight_backward", C.c_void_p),
        ("sizes", C.c_void_p), ("dst_local_id", C.c_void_p), ("csr_edge_id", C.c_void_p),
        ("omit_map", C.c_void_p), ("omit_key", C.c_uint32), ("omit_loc", C.c_void_p),
        ("omit_row", C.c_void_p),
        ("sizes_host", C.c_void_p),
    ]


_lib = None


def lib() -> C.CDLL:
    """Load libnts_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (there is no CPU fallback for the HIP path)")
    L = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    P, U32, U64, I, F = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_float
    sig = {
        "nts_hip_abi_version": ([], I),
        "nts_hip_last_error": ([], C.c_char_p),
        "nts_hip_ctx_create": ([C.POINTER(P), I, P, U64], I),
        "nts_hip_ctx_destroy": ([P], I),
        "nts_hip_ctx_set_stream": ([P, P], I),
        "nts_hip_ctx_get_stream": ([P], P),
        "nts_hip_ctx_set_gemm_mode": ([P, I], I),
        "nts_hip_ctx_get_gemm_mode": ([P], I),
        "nts_hip_ctx_reserve": ([P, U64, U64], I),
        "nts_hip_rng_seed": ([P, U64], I),
        "nts_hip_mt_budget_scale": ([P, C.c_double], I),
        "nts_hip_mt_checkpoint": ([P, P], I),
        "nts_hip_mt_rewind": ([P, P], I),
        "nts_hip_rng_state": ([P, P], I),
        "nts_hip_degrees": ([P, P, P, U64, U64, P, P], I),
        "nts_hip_build_csc": ([P, P, P, U64, U64, P, P], I),
        "nts_hip_sample_layer": ([P, C.POINTER(GraphDev), I, I, U64, I, I, C.POINTER(SampCSCDev)], I),
        "nts_hip_gather_rows": ([P, P, U64, P, P, U32, U32, P, U64], I),
        "nts_hip_gather_labels": ([P, P, P, P, U32, P], I),
        "nts_hip_spmm_csc_fwd": ([P, P, P, P, P, U32, P, U64, P, U32, P, U64], I),
        "nts_hip_spmm_csc_fwd_act": ([P, P, P, P, P, U32, P, U64, U32, P, U64, F, U64, U64], I),
        "nts_hip_spmm_csr_bwd_masked": ([P, P, P, P, P, U32, P, U64, P, U64, F, U32, P, U64], I),
        "nts_hip_spmm_csr_bwd_postmask": ([P, P, P, P, P, U32, P, U64, P, U64, F, U32, P, U64], I),
        "nts_hip_act_bits_words": ([U32], U32),
        "nts_hip_spmm_csc_fwd_act_bits": ([P, P, P, P, P, U32, P, U64, U32, P, U64, F, U64, U64, P], I),
        "nts_hip_spmm_csr_bwd_postmask_bits": ([P, P, P, P, P, U32, P, U64, P, F, U32, P, U64], I),
        "nts_hip_act_backward": ([P, U32, U32, P, U64, P, U64, F, P, U64], I),
        "nts_hip_presample_counts": ([P, C.POINTER(GraphDev), P, U32, I, P, P], I),
        "nts_hip_presample_select": ([P, P, U64, F, P, P], I),
        "nts_hip_pd_set_cache": ([P, P, U32, U32, P, P], I),
        "nts_hip_pd_load_share": ([P, P, P, U32, P, U64, U32, P, U64], I),
        "nts_hip_relu_dropout_f32": ([P, U32, U32, P, U64, F, U64, U64, P, U64], I),
        "nts_hip_gemm_gather_f32": ([P, I, I, I, P, U64, P, P, U64, P, U64], I),
        "nts_hip_gemm_tn_gather_f32": ([P, I, I, I, P, U64, P, P, U64, P, U64], I),
        "nts_hip_h2_split_rows": ([P, U64, U32, P, U64, U32, P, U64, P], I),
        "nts_hip_gemm_h2_gather": ([P, I, I, I, I, P, U64, P, P, P, U64, I, P, U64, F, U64, U64], I),
        "nts_hip_gemm_h2_tn_gather": ([P, I, I, I, P, U64, P, P, P, U64, P, U64, F, P, U64], I),
        "nts_hip_h2_split_rows_planar": ([P, U64, U32, P, U64, U32, P, U64, P], I),
        "nts_hip_gemm_h2p_tn_gather": ([P, I, I, I, P, U64, I, P, P, P, U64, P, U64], I),
        "nts_hip_gemm_h2p_tn_gather_cm": ([P, I, I, I, P, U64, I, P, P, P, U64, P, U64, P, U32], I),
        "nts_hip_gemm_h2p_gather": ([P, I, I, I, I, P, U64, P, P, P, U64, I, P, U64, F, U64, U64], I),
        "nts_hip_spmm_csr_bwd": ([P, P, P, P, P, U32, P, U64, U32, P, U64], I),
        "nts_hip_spmm_csr_bwd_colmax": ([P, P, P, P, P, U32, P, U64, U32, P, U64, P, P, P], I),
        "nts_hip_csr_bwd_colmax_rows_per_part": ([U32], U32),
        "nts_hip_gemm_h2d_act": ([P, I, I, I, I, P, U64, P, U64, P, U64, F, U64, U64, P, U64, P], I),
        "nts_hip_spmm_csc_bwd_atomic": ([P, P, P, P, P, U32, P, U64, U32, P, U64], I),
        "nts_hip_gemm_f32": ([P, I, I, I, I, P, U64, P, U64, P, U64], I),
        "nts_hip_gemm_relu_dropout_f32": ([P, I, I, I, P, U64, P, U64, P, U64, F, U64, U64], I),
        "nts_hip_gemm_tn_masked_f32": ([P, I, I, I, P, U64, P, U64, P, U64, F, P, U64], I),
        "nts_hip_linear_xent_fwd": ([P, P, U64, I, I, P, I, P, P, P], I),
        "nts_hip_linear_xent_bwd": ([P, P, U64, I, I, P, I, P, P, P, P], I),
        "nts_hip_linear_xent_train": ([P, P, U64, I, I, P, I, P, P, P, P, P], I),
        "nts_hip_adam": ([P, P, P, P, P, U64, F, F, F, F, F, F, F, I], I),
        "nts_hip_comm_unique_id": ([P], I),
        "nts_hip_comm_init": ([C.POINTER(P), I, I, P, I], I),
        "nts_hip_comm_destroy": ([P], I),
        "nts_hip_comm_count": ([P, C.POINTER(I), C.POINTER(I)], I),
        "nts_hip_allreduce_sum_f32": ([P, P, U64, P], I),
        "nts_hip_broadcast_f32": ([P, P, U64, I, P], I),
        "nts_hip_cache_select": ([P, P, U64, U64, P, P], I),
        "nts_hip_host_alloc": ([U64, C.POINTER(P)], I),
        "nts_hip_host_free": ([P], I),
        "nts_hip_host_device_pointer": ([P, C.POINTER(P)], I),
        "nts_hip_gather_rows_cached": ([P, P, U64, P, P, U64, P, P, U32, U32, P, U64], I),
        "nts_hip_spmm_csc_fwd_cached": ([P, P, P, P, P, U32, P, U64, P, P, U64, I, P, U32, P, U64], I),
        "nts_hip_stage_uncached_rows": ([P, P, P, U64, P, P, U32, U32, P, U64], I),
        "nts_hip_gat_forward": ([P, P, P, P, U32, P, U64, U32, P, P, P, P, U64], I),
        "nts_hip_gat_backward": ([P, P, P, P, U32, P, P, P, U32, P, U64, U32, P, P, P, P, U64,
                                  P, U64, P, P, P, U64, P, U64, P], I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.nts_hip_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI {L.nts_hip_abi_version()}, the bindings expect "
                          f"{ABI_VERSION}: rebuild it")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != NTS_OK:
        msg = lib().nts_hip_last_error().decode(errors="replace")
        raise RuntimeError(f"nts_hip error {rc}: {msg}")


def ptr(t) -> int | None:
    """Raw device/host pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()
