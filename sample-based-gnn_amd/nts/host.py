"""Python access to the C++ host layer (nts/host/*.cpp, built in-tree).

`ext()` loads nts/lib/host_build/nts_host_ext.so — it raises when the build is
missing; nothing here falls back to a CPU implementation.
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import pathlib

import torch  # noqa: F401  (torch's HIP runtime first)

from . import _abi

_HERE = pathlib.Path(__file__).resolve().parent
EXT_PATH = _HERE / "lib" / "host_build" / "nts_host_ext.so"
_ext = None


def ext():
    global _ext
    if _ext is None:
        if not EXT_PATH.exists():
            raise ImportError(f"{EXT_PATH} missing: run __graft_entry__.build()")
        _abi.lib()  # libnts_hip.so first (RTLD_GLOBAL)
        loader = importlib.machinery.ExtensionFileLoader("nts_host_ext", str(EXT_PATH))
        spec = importlib.util.spec_from_loader("nts_host_ext", loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _ext = mod
    return _ext


def gcn_config(layers, fanout, batch_size, learn_rate=0.01, weight_decay=1e-4, drop_rate=0.5,
               rng_mode=_abi.NTS_RNG_PHILOX, weight="sum", fused_gather=True,
               bias_correction=False, deterministic_backward=True, shuffle=True, profile=False,
               seed=2000, hip_gemm=True, pipeline=True, transform_first=-1,
               early_aggregate=True, sampler_priority=2, fuse_activation=True,
               fuse_loss=True, sampler_cus=0, sampler_gate=0, pad_features=True, cache_rate=-1.0,
               up_degree=False, gat=False, pd_cache=False, pd_rate=0.2, pd_super_batch=4,
               gemm="split3", overlap_allreduce=-1, pair_table=0, sample_gpu=False):
    E = ext()
    c = E.GCNConfig()
    c.layer_size = list(layers)
    c.fanout = list(fanout)
    c.batch_size = int(batch_size)
    c.learn_rate = float(learn_rate)
    c.weight_decay = float(weight_decay)
    c.drop_rate = float(drop_rate)
    c.rng_mode = int(rng_mode)
    c.sample_gpu = bool(sample_gpu)
    c.weight_type = {"sum": E.WeightType.Sum, "mean": E.WeightType.Mean,
                     "mean-sampled": E.WeightType.MeanSampled,
                     "none": getattr(E.WeightType, "None")}[weight]
    c.fused_gather = bool(fused_gather)
    c.bias_correction = bool(bias_correction)
    c.deterministic_backward = bool(deterministic_backward)
    c.hip_gemm = bool(hip_gemm)
    c.pipeline = bool(pipeline)
    c.transform_first = int(transform_first)
    c.gemm_mode = {"f32": _abi.NTS_GEMM_F32, "split3": _abi.NTS_GEMM_SPLIT3}[gemm]
    c.overlap_allreduce = int(overlap_allreduce)
    c.pair_table = int(pair_table)
    c.early_aggregate = bool(early_aggregate)
    c.sampler_priority = int(sampler_priority)
    c.fuse_activation = bool(fuse_activation)
    c.fuse_loss = bool(fuse_loss)
    c.sampler_cus = int(sampler_cus)
    c.sampler_gate = int(sampler_gate)
    c.pad_features = bool(pad_features)
    c.cache_rate = float(cache_rate)
    c.up_degree = bool(up_degree)
    c.gat = bool(gat)
    c.pd_cache = bool(pd_cache)
    c.pd_rate = float(pd_rate)
    c.pd_super_batch = int(pd_super_batch)
    c.shuffle = bool(shuffle)
    c.profile = bool(profile)
    c.seed = int(seed)
    return c
