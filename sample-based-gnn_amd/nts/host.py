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
               seed=2000, hip_gemm=True, pipeline=True, fuse_linear=False,
               early_aggregate=True, sampler_priority=True, fuse_activation=True,
               fuse_loss=True, sampler_cus=0, pad_features=True, cache_rate=-1.0,
               up_degree=False, gat=False):
    E = ext()
    c = E.GCNConfig()
    c.layer_size = list(layers)
    c.fanout = list(fanout)
    c.batch_size = int(batch_size)
    c.learn_rate = float(learn_rate)
    c.weight_decay = float(weight_decay)
    c.drop_rate = float(drop_rate)
    c.rng_mode = int(rng_mode)
    c.weight_type = {"sum": E.WeightType.Sum, "mean": E.WeightType.Mean,
                     "none": getattr(E.WeightType, "None")}[weight]
    c.fused_gather = bool(fused_gather)
    c.bias_correction = bool(bias_correction)
    c.deterministic_backward = bool(deterministic_backward)
    c.hip_gemm = bool(hip_gemm)
    c.pipeline = bool(pipeline)
    c.fuse_linear = bool(fuse_linear)
    c.early_aggregate = bool(early_aggregate)
    c.sampler_priority = bool(sampler_priority)
    c.fuse_activation = bool(fuse_activation)
    c.fuse_loss = bool(fuse_loss)
    c.sampler_cus = int(sampler_cus)
    c.pad_features = bool(pad_features)
    c.cache_rate = float(cache_rate)
    c.up_degree = bool(up_degree)
    c.gat = bool(gat)
    c.shuffle = bool(shuffle)
    c.profile = bool(profile)
    c.seed = int(seed)
    return c


def smoke_step(dev: torch.device) -> None:
    """Tiny end-to-end check of the host layer on the GPU: a 2-layer GCN on a
    small synthetic graph — eval forward vs the CPU oracle, then training steps."""
    import numpy as np

    from oracle import oracle as orc

    from . import synthetic

    E = ext()
    g = synthetic.chung_lu(3000, 60000, 10.0, device=dev, seed=1)
    G = E.FullyRepGraph.from_edges(g.src, g.dst, g.n_vertices)
    F_dim, C = 48, 5
    feat = synthetic.features(g.n_vertices, F_dim, device=dev)
    labels, masks = synthetic.labels_masks(g.n_vertices, C, device=dev)
    train = torch.nonzero(masks == 0).flatten().to(torch.int32).cpu()
    cfg = gcn_config([F_dim, 16, C], [10, 5], 128, drop_rate=0.0)
    drv = E.GCN_SAMPLE_ALLGPU_impl(G, feat, labels, train, cfg)
    seeds = torch.arange(0, 256, dtype=torch.int32)
    acts = drv.forward_eval(seeds, 0)
    # oracle: same graph, PHILOX stream (batch_seq 0), CPU fuse + torch CPU GEMM
    src = g.src.cpu().numpy().view(np.uint32)
    dst = g.dst.cpu().numpy().view(np.uint32)
    col, rows = orc.build_csc(g.n_vertices, src, dst)
    od, idg = orc.degrees(g.n_vertices, src, dst)
    o = orc.Sampler(col, rows, idg, od, [10, 5], seed=2000, rng_mode=orc.RNG_PHILOX,
                    order_mode=orc.ORDER_DRAW)
    l0, l1 = o.sample(seeds.numpy().astype(np.uint32))
    W = [w.cpu() for w in drv.weights()]
    X0 = orc.get_feature(l1["source"], feat.cpu().numpy())
    Y0 = orc.fuse_fwd(l1, X0, od, idg)
    X1 = torch.relu(torch.from_numpy(Y0) @ W[0])
    Y1 = orc.fuse_fwd(l0, X1.numpy(), od, idg)
    X2 = (torch.from_numpy(Y1) @ W[1]).log_softmax(1)
    assert torch.equal(acts[0].cpu(), torch.from_numpy(Y0)), "Y0 differs"
    for got, ref in ((acts[1], X1), (acts[2], torch.from_numpy(Y1)), (acts[3], X2)):
        torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=1e-4)
    for _ in range(3):
        drv.train_batch()
    drv.synchronize()
    assert torch.isfinite(drv.loss).item()
