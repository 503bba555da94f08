#!/usr/bin/env python3
"""Headline benchmark: sampled-edges/sec + epoch time of 2-hop GCN training on a
Reddit-shaped synthetic graph (BASELINE.json configs[1]: GCN_SAMPLE_GPU-style
602-128-41, fanout 25-10, batch 10,000, V=232,965, E~114.8M incl. self-loops).

A step = one mini-batch of the hot path, everything on the GPU: GPU neighbour
sampling (2 hops) -> label gather -> fused feature gather + hop-1 aggregation
-> GEMM/ReLU/dropout -> hop-0 aggregation -> GEMM/log_softmax -> NLL ->
backward (CSR transpose aggregation + GEMM grads) -> [RCCL all-reduce] -> Adam.

value = sampled edges of all ranks in the K timed steps / max-over-ranks wall
time.  Inputs are resident in HBM before the timed region.

Multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
(one process per GPU, seeds sharded, one fused RCCL SUM all-reduce per step).
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "sample-based-gnn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "sampled-edges/sec + epoch time, 2-hop GCN on Reddit-shaped graph @1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--shape", default="reddit")
    p.add_argument("--batch", type=int, default=10000)
    p.add_argument("--fanout", default="25-10")
    p.add_argument("--hidden", type=int, default=128)
    p.add_argument("--layers", default=None,
                   help="layer widths a-b-...-c (default: F-hidden-classes of the shape)")
    p.add_argument("--weight", default="sum", choices=["sum", "mean"],
                   help="edge weights: GCN sum (default) or GraphSAGE mean")
    p.add_argument("--no-fused-gather", action="store_true")
    p.add_argument("--no-pipeline", action="store_true", help="sample on the training stream")
    p.add_argument("--no-hip-gemm", action="store_true", help="layer GEMMs through torch.matmul")
    p.add_argument("--early-agg", action="store_true",
                   help="issue the bottom aggregation behind the sampler on the sampling stream")
    p.add_argument("--no-priority", action="store_true", help="sampler stream at normal priority")
    p.add_argument("--model", default="gcn", choices=["gcn", "gat"],
                   help="gcn (headline) or gat (GAT_SAMPLE_ALL_GPU-style attention layers)")
    p.add_argument("--atomic-backward", action="store_true",
                   help="graph-op backward by atomic CSC scatter (no CSR transpose in the "
                        "sampler; nondeterministic sums)")
    p.add_argument("--cache-rate", type=float, default=-1.0,
                   help="feature table in pinned host memory with this fraction of the "
                        "highest-degree rows cached in HBM (GS_SAMPLE_PD_CACHE placement); "
                        "default: whole table in HBM")
    p.add_argument("--no-fuse-act", action="store_true",
                   help="relu/dropout as torch ops instead of the GEMM epilogue")
    p.add_argument("--sampler-cus", type=int, default=0,
                   help="CUs reserved for the pipelined sampler stream (0: no partition)")
    p.add_argument("--no-pad-features", action="store_true",
                   help="gather from the feature table as given (no 128-byte row pitch copy)")
    p.add_argument("--no-fuse-loss", action="store_true",
                   help="output layer + loss as libtorch ops instead of the fused kernels")
    p.add_argument("--fuse-linear", action="store_true",
                   help="bottom layer: aggregation and first GEMM in one kernel")
    p.add_argument("--cpu-baseline-steps", type=int, default=10)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    p.add_argument("--no-epoch", action="store_true", help="skip the timed full epoch")
    p.add_argument("--scale", type=float, default=1.0)
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # NTS_BENCH_SHARE_GPU=1: every rank on device 0 (rehearsing the DP path on a
    # one-GPU box; the numbers are then not a scaling measurement)
    if os.environ.get("NTS_BENCH_SHARE_GPU") == "1":
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    from nts import host, synthetic
    from nts import _abi
    E = host.ext()

    # ---- inputs resident in HBM -------------------------------------------------
    t0 = time.time()
    g, F_dim, C = synthetic.shaped(args.shape, device=dev, scale=args.scale)
    G = E.FullyRepGraph.from_edges(g.src, g.dst, g.n_vertices)
    V, En = g.n_vertices, g.n_edges
    feat = synthetic.features(V, F_dim, device=dev)
    labels, masks = synthetic.labels_masks(V, C, device=dev)
    train = torch.nonzero(masks == 0).flatten().to(torch.int32).cpu()
    # DP: contiguous equal slices (remainder dropped so every rank runs the same
    # number of steps; the reference gives it to the last GPU,
    # toolkits/GCN_SAMPLE_ALL_MULTI.hpp:564-575)
    from nts import dist as ndist
    train = ndist.shard_nids(train, world, rank)
    log(f"[bench] graph {args.shape}: V={V} E={En} F={F_dim} C={C}  ready in {time.time()-t0:.1f}s")
    src_host = g.src.cpu().numpy().view(np.uint32) if (rank == 0 and world == 1 and not args.no_cpu_baseline) else None
    dst_host = g.dst.cpu().numpy().view(np.uint32) if src_host is not None else None
    del g

    comm = ndist.make_communicator(E, world, rank, local_rank)

    fan = [int(x) for x in args.fanout.split("-")]
    layers = ([int(x) for x in args.layers.split("-")] if args.layers else [F_dim, args.hidden, C])
    if layers[0] != F_dim or len(layers) != len(fan) + 1:
        raise SystemExit(f"--layers must start at the feature width {F_dim} and have one more "
                         f"entry than --fanout")
    cfg = host.gcn_config(layers, fan, args.batch, learn_rate=0.001, weight_decay=1e-4,
                          drop_rate=0.5, rng_mode=_abi.NTS_RNG_PHILOX, weight=args.weight,
                          fused_gather=not args.no_fused_gather, profile=True,
                          pipeline=not args.no_pipeline, hip_gemm=not args.no_hip_gemm,
                          fuse_linear=args.fuse_linear, early_aggregate=args.early_agg,
                          sampler_priority=not args.no_priority,
                          fuse_activation=not args.no_fuse_act,
                          fuse_loss=not args.no_fuse_loss, sampler_cus=args.sampler_cus,
                          pad_features=not args.no_pad_features, cache_rate=args.cache_rate,
                          deterministic_backward=not args.atomic_backward,
                          gat=args.model == "gat")
    fused_linear = (not args.no_fused_gather and args.fuse_linear and not args.no_hip_gemm
                    and not args.early_agg and layers[1] <= 128)
    agg_kernel = ("k_agg_gemm" if fused_linear else "k_spmm_gather")
    if args.model == "gat":
        agg_kernel = "k_gat_fwd"  # not timed by the driver's bottom-aggregation events
    drv = E.GCN_SAMPLE_ALLGPU_impl(G, feat, labels, train, cfg, comm)

    def step():
        if not drv.sample_not_finished():
            drv.restart()
        drv.train_batch()

    for _ in range(args.warmup):
        step()
    drv.synchronize()
    drv.reset_stats()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drv.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    agg_ms = drv.resolve_profile()
    edges = float(drv.batch_edges)
    agg_bytes = float(drv.agg_bytes)
    agg_calls = int(drv.agg_calls)
    sample_s = float(drv.sample_time)
    train_host_s = float(drv.train_time)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed, edges], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, edges = float(mx[0]), float(t[1])

    # sizes of the last timed batch (before the epoch run replaces them)
    layer_sizes = [{"v": int(l["v_size"]), "src": int(l["src_size"]), "e": int(l["e_size"])}
                   for l in drv.last_layers]
    epoch_s = None
    if not args.no_epoch:
        drv.restart()
        barrier()
        te = time.perf_counter()
        drv.run_epoch()
        drv.synchronize()
        barrier()
        epoch_s = time.perf_counter() - te
        drv.resolve_profile()
        if world > 1:
            import torch.distributed as dist
            t = torch.tensor([epoch_s], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            epoch_s = float(t[0])

    value = edges / elapsed
    agg_avg_ms = agg_ms / max(agg_calls, 1)
    achieved = (agg_bytes / max(agg_calls, 1)) / (agg_avg_ms * 1e-3) / 1e9 if agg_calls else None
    n_train_per_gpu = int(train.numel())
    batches_per_epoch = -(-n_train_per_gpu // args.batch)

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "sampled-edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic Chung-Lu power-law graph (seed 2024), N(0,1) fp32 features (seed 7), uniform labels",
        "config": {
            "workload": (f"{'GAT_SAMPLE_ALL_GPU' if args.model == 'gat' else ('GS' if args.weight == 'mean' else 'GCN') + '_SAMPLE_ALLGPU'}-style "
                         f"{len(layers) - 1}-layer {'GAT' if args.model == 'gat' else ('GraphSAGE (mean)' if args.weight == 'mean' else 'GCN')} "
                         f"{'-'.join(map(str, layers))}, fanout "
                         f"{args.fanout}, batch {args.batch}/GPU, {args.shape}-shaped synthetic "
                         f"(V={V}, E={En}); GPU sampler (Philox"
                         f"{', pipelined' if not args.no_pipeline else ''}) + fused gather/aggregation"
                         f"{' (issued behind the sampler)' if args.early_agg and not args.no_fused_gather else ''}"
                         f"{' + layer-1 GEMM' if fused_linear else ''} + "
                         f"{'torch' if args.no_hip_gemm else 'MFMA'} GEMM + fused Adam"
                         + (f"; features in pinned host memory, {args.cache_rate:.0%} of rows "
                            f"(highest degree) cached in HBM" if args.cache_rate >= 0 else "")),
            "global_batch": args.batch * world,
            "parallelism": f"dp{world}",
            "fanout": args.fanout,
            "epoch_time_s": epoch_s if epoch_s is not None else elapsed / args.steps * batches_per_epoch,
            "epoch_time_kind": ("measured: one full epoch over this rank's training shard, "
                                "after the timed steps" if epoch_s is not None
                                else "ms_per_step x batches/epoch"),
            "batches_per_epoch_per_gpu": batches_per_epoch,
            "sampler_s_per_step": sample_s / args.steps,
            "host_train_issue_s_per_step": train_host_s / args.steps,
            "layer_sizes_top_down": layer_sizes,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": agg_kernel + (" (feature gather + hop-1 aggregation + layer-1 GEMM)" if fused_linear
                                    else " (fused feature gather + hop-1 aggregation)"),
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": None,
            "avg_launch_ms": agg_avg_ms,
            "algorithmic_bytes_per_launch": agg_bytes / max(agg_calls, 1),
        },
    }
    # HBM traffic of the dominant kernel from the newest committed PMC pass
    # (profiles/pmc_<tag>.json, FETCH_SIZE x 2 + WRITE_SIZE per launch) — valid for
    # the default workload only
    pmcs = sorted((ROOT / "profiles").glob("pmc_*.json"))
    default_shape = (args.shape == "reddit" and args.batch == 10000 and args.fanout == "25-10"
                     and layers == [602, 128, 41] and world == 1 and args.cache_rate < 0)
    if pmcs and default_shape:
        try:
            info = json.loads(pmcs[-1].read_text())
            if info.get("kernel", "").split("<")[0].split("::")[-1] == agg_kernel:
                tb = float(info["hbm_bytes_per_launch"])
                result["roofline"]["traffic"] = tb
                result["roofline"]["traffic_source"] = pmcs[-1].name
                # actual HBM bytes moved per launch / this run's launch time
                result["roofline"]["traffic_GBs"] = tb / (agg_avg_ms * 1e-3) / 1e9
                result["roofline"]["traffic_frac"] = result["roofline"]["traffic_GBs"] / HBM_PEAK_GBS
        except Exception:
            pass

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, G, feat, labels, train, fan, layers,
                                              src_host, dst_host, V)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def cpu_baseline(args, G, feat, labels, train, fan, layers, src_host, dst_host, V):
    """The reference CPU path restated (oracle/ref_cpu.cpp, GCN_CPU_SAMPLE.hpp:194-256)
    timed on this host: sample_fast (OpenMP, thread-local mt19937), get_feature,
    MiniBatchFuseOp fwd/bwd (CAS backward), libtorch CPU GEMM + Adam."""
    from oracle import oracle as orc
    threads = max(1, args.cpu_threads)
    torch.set_num_threads(threads)
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    in_d = G.in_degree.cpu().numpy().view(np.uint32)
    out_d = G.out_degree.cpu().numpy().view(np.uint32)
    feat_h = feat.cpu().numpy()
    lab_h = labels.cpu()
    s = orc.Sampler(col, rows, in_d, out_d, fan, seed=2000, rng_mode=orc.RNG_MT_LEMIRE,
                    order_mode=orc.ORDER_UNORDERED_MAP)
    gen = torch.Generator().manual_seed(0)
    W = [torch.empty(a, b).uniform_(-(6 / (a + b)) ** 0.5, (6 / (a + b)) ** 0.5, generator=gen).requires_grad_()
         for a, b in zip(layers[:-1], layers[1:])]
    M = [torch.zeros_like(w) for w in W]
    Vv = [torch.zeros_like(w) for w in W]
    ids = train.numpy().astype(np.uint32)
    total_edges, total_t = 0, 0.0
    for it in range(max(1, args.cpu_baseline_steps)):
        seeds = ids[it * args.batch:(it + 1) * args.batch]
        t0 = time.perf_counter()
        l0, l1 = s.sample(seeds, it, orc.W_SUM, True, threads)
        X0 = orc.get_feature(l1["source"], feat_h, threads)
        Y0 = torch.from_numpy(orc.fuse_fwd(l1, X0, out_d, in_d, threads=threads))
        X1 = torch.dropout(torch.relu(Y0 @ W[0]), 0.5, True)
        Y1 = torch.from_numpy(orc.fuse_fwd(l0, X1.detach().numpy(), out_d, in_d, threads=threads))
        Y1.requires_grad_()
        X2 = Y1 @ W[1]
        tgt = lab_h[torch.from_numpy(l0["destination"].astype(np.int64))]
        loss = torch.nn.functional.nll_loss(X2.log_softmax(1), tgt)
        loss.backward()
        gX1 = orc.fuse_bwd(l0, Y1.grad.numpy(), out_d, in_d, threads=threads)
        X1.backward(torch.from_numpy(gX1))
        with torch.no_grad():  # learnC2C_with_decay_Adam
            for i, w in enumerate(W):
                wg = w.grad + 1e-4 * w
                M[i] = 0.9 * M[i] + 0.1 * wg
                Vv[i] = 0.999 * Vv[i] + 0.001 * wg * wg
                w -= 0.001 * (M[i] / 0.1) / (torch.sqrt(Vv[i] / 0.001) + 1e-9)
                w.grad = None
        total_t += time.perf_counter() - t0
        total_edges += l0["e_size"] + l1["e_size"]
    return {
        "value": total_edges / total_t,
        "unit": "sampled-edges/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{max(1, args.cpu_baseline_steps)} GCN_CPU_SAMPLE training step(s) of batch "
                   f"{args.batch} on the same graph ({total_edges} sampled edges, {total_t:.1f}s), "
                   f"OpenMP {threads} threads, oracle/ref_cpu.cpp -O3 x86-64-v3 + torch CPU"),
    }


if __name__ == "__main__":
    main()
