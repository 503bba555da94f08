#!/usr/bin/env python3
"""Headline benchmark: sampled-edges/sec + epoch time of 2-hop GCN training on a
Reddit-shaped synthetic graph (BASELINE.json configs[1]: GCN_SAMPLE_GPU-style
602-128-41, fanout 25-10, batch 10,000, V=232,965, E~114.8M incl. self-loops).

A step = one mini-batch of the hot path, everything on the GPU: GPU neighbour
sampling (2 hops, on its own stream, batches ahead) -> label gather -> bottom
layer (transform-first: row-gathered GEMM X[src] W0, then the aggregation with
relu/dropout fused) -> hop-0 aggregation -> output layer + log_softmax + NLL ->
backward (CSR transpose aggregations, gathered weight-gradient GEMM) ->
[RCCL all-reduce] -> Adam.

value = sampled edges of all ranks in the K timed steps / max-over-ranks wall
time.  Inputs are resident in HBM before the timed region.

Multi-GPU: `python bench.py --gpus N` starts `python -m torch.distributed.run
--nproc-per-node N bench.py --gpus N ...` as a child process (before anything
touches the GPU), relays rank 0's JSON line and exits with the child's status;
launched that way or by the driver's own torch.distributed.run, every rank
checks WORLD_SIZE == --gpus, and the line carries `rccl_ranks` as RCCL reports
it (ncclCommCount).  One process per GPU, seeds sharded, one fused RCCL SUM
all-reduce per step (toolkits/GCN_SAMPLE_ALL_MULTI.hpp:89-113,367-377).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import pathlib
import subprocess
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "sample-based-gnn_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TF = 157.3  # MI355X fp32 matrix peak (MI355X_MICROARCH.md)
F16_MFMA_PEAK_TF = 2500.0  # MI355X dense f16/bf16 matrix peak (MI355X_MICROARCH.md)
SHAPE_NAMES = {"reddit": "Reddit", "products": "ogbn-products", "papers100m": "ogbn-papers100M",
               "tiny": "tiny"}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_quota():
    """CPUs this job may use by its cgroup's CFS quota (v2 cpu.max, v1
    cfs_quota_us / cfs_period_us); None when there is no quota."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_share() -> dict:
    """The inputs of the CPU-baseline thread rule, recorded in the bench line."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = None
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_quota": cpu_quota(),
            "omp_num_threads": int(omp) if omp and omp.isdigit() else None}


def default_cpu_threads() -> int:
    """The reference's sampler uses nproc-1 threads (core/FullyRepGraph.hpp:49),
    capped by what this job may use: the affinity mask, the cgroup CPU quota
    and the job's declared CPU share (OMP_NUM_THREADS; 16 per GPU on the GPU
    box, where nproc shows the whole machine)."""
    s = cpu_share()
    n = (s["nproc"] or 2) - 1
    for cap in (s["affinity_cpus"], s["cpu_quota"], s["omp_num_threads"]):
        if cap:
            n = min(n, max(1, int(cap)))
    return max(1, n)


# the NTS_* variables something on the measured path still reads: the
# library (a launch-trace debug aid and the two MT19937 walker selections),
# the host extension (two host-side timing aids), this script (an A/B library
# path and the shared-GPU rehearsal); every other knob is a compile-time flag
READ_ENV = ("NTS_LAUNCH_TRACE", "NTS_MT_SERIAL", "NTS_MT_CHUNKED", "NTS_HOST_PROFILE", "NTS_TIMELINE",
            "NTS_HIP_LIB", "NTS_BENCH_SHARE_GPU")


def nts_env() -> dict:
    """The NTS_* variables of this run that are read (recorded in
    profile_meta), and under "ignored" the names of any set that nothing reads
    any more (former A/B knobs, now `make variant` flags)."""
    env = {k: v for k, v in sorted(os.environ.items()) if k in READ_ENV}
    ignored = sorted(k for k in os.environ if k.startswith("NTS_") and k not in READ_ENV)
    if ignored:
        env["ignored"] = ignored
    return env


def diag_env() -> list:
    """NTS_*DIAG* variables: diagnostics that skip work or give wrong results;
    a bench line measured under one is invalid, so bench.py refuses to run."""
    return sorted(k for k in os.environ if k.startswith("NTS_") and "DIAG" in k)


def free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv: list, n: int) -> int:
    """`bench.py --gpus N` without a launcher: run `torch.distributed.run
    --nproc-per-node N bench.py ...` as a CHILD process (this process has not
    touched the GPU and never execs), relay rank 0's JSON line, and return the
    child's exit status — non-zero also when no line came back or its n_gpus
    is not N."""
    shared = os.environ.get("NTS_BENCH_SHARE_GPU") == "1"
    if not shared and "--launch-selftest" not in argv:
        have = torch.cuda.device_count()  # counts devices without initialising HIP
        if have < n:
            print(f"[bench] --gpus {n} but this node has {have} GPU(s)", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           str(ROOT / "bench.py"), *argv]
    env = dict(os.environ, PYTHONUNBUFFERED="1", MASTER_ADDR="127.0.0.1")
    log(f"[bench] launching {n} ranks: {' '.join(cmd)}")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    line = None
    for out in p.stdout:
        try:
            obj = json.loads(out)
        except ValueError:
            obj = None
        if isinstance(obj, dict) and "metric" in obj:
            line = obj
        else:
            sys.stderr.write(out)
            sys.stderr.flush()
    rc = p.wait()
    if rc != 0:
        print(f"[bench] the {n}-rank run exited with {rc}", file=sys.stderr)
        return rc
    if line is None or line.get("n_gpus") != n:
        print(f"[bench] the {n}-rank run reported no line for {n} ranks: {line}", file=sys.stderr)
        return 1
    line.setdefault("config", {})["launcher"] = (
        f"bench.py --gpus {n} -> child `python -m torch.distributed.run --nproc-per-node {n}`")
    print(json.dumps(line), flush=True)
    return 0


def launch_selftest(world: int, rank: int) -> None:
    """--launch-selftest: the launcher's control flow without a GPU — every
    rank joins a gloo group and rank 0 prints a line with the ranks that
    answered (tests/test_bench.py)."""
    import torch
    import torch.distributed as dist
    ar_us = None
    if world > 1:
        dist.init_process_group("gloo")
        ranks = [None] * world
        dist.all_gather_object(ranks, rank)
        # the line's gradient-exchange fields, as the real run reports them:
        # one SUM all-reduce of the C2 bucket (602*128 + 128*41 floats) per
        # step, host wall time, max over ranks
        bucket = torch.ones(602 * 128 + 128 * 41)
        t = []
        for _ in range(3):
            t0 = time.perf_counter()
            dist.all_reduce(bucket)
            t.append(time.perf_counter() - t0)
        m = torch.tensor([1e6 * sum(t) / len(t)], dtype=torch.float64)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        ar_us = float(m[0])
        dist.destroy_process_group()
    else:
        ranks = [0]
    if rank == 0:
        print(json.dumps({"metric": "launch-selftest", "value": 0.0, "n_gpus": world,
                          "ranks": ranks, "rccl_ranks": None,
                          "config": {"allreduce_us_per_step": ar_us,
                                     "allreduce_timing": {"how": "host wall time (gloo, CPU)"}}}),
              flush=True)


# flags of the parent run that a secondary child must not inherit: the
# secondary machinery itself, the launcher, the CPU baseline and the extra
# measurements only the headline run makes (value-taking flags map to True)
_CHILD_DROP = {"--secondary": False, "--no-secondary-exact": False, "--no-secondary-mt": False,
               "--no-secondary-af": False, "--gpus": True, "--no-cpu-baseline": False,
               "--cpu-threads": True, "--cpu-max-steps": True, "--cpu-o0-steps": True,
               "--epochs": True, "--sampler-batches": True, "--no-interference-probe": False,
               "--launch-selftest": False}


def child_argv(argv: list, overrides: dict) -> list:
    """A secondary child's argv: the parent's own workload flags (argv, as
    given on the command line) minus `_CHILD_DROP`, with every flag in
    `overrides` ({"--rng": "mt", ...}) replaced, then `--secondary`."""
    out, i = [], 0
    while i < len(argv):
        a = argv[i]
        key, has_eq = (a.split("=", 1)[0], True) if a.startswith("--") and "=" in a else (a, False)
        takes = _CHILD_DROP.get(key)
        if key in overrides:
            takes = True
        if takes is None:
            out.append(a)
        elif takes and not has_eq:
            i += 1  # drop the flag's value too
        i += 1
    for k, v in overrides.items():
        out += [k, str(v)]
    return out + ["--secondary"]


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
    p.add_argument("--weight", default="sum", choices=["sum", "mean", "mean-sampled"],
                   help="edge weights: GCN sum (default), GraphSAGE mean (CPU formula) or the "
                        "reference GPU kernel's mean (by sampled count)")
    p.add_argument("--transform-first", type=int, default=-1, choices=[-1, 0, 1],
                   help="bottom layer order: 1 A(XW), 0 (AX)W (the reference's), -1 auto")
    p.add_argument("--gemm", default="split3", choices=["f32", "split3"],
                   help="layer GEMM arithmetic: f32 = fp32-input MFMA; split3 = fp32 operands "
                        "split exactly into three bf16 pieces, six piece products on the bf16 "
                        "MFMA (fp32-accurate, csrc/gemm3.hip)")
    p.add_argument("--pair-table", type=int, default=0, choices=[0, 1, 2, 3],
                   help="transform-first GEMMs on the feature table's f16 pair table "
                        "(csrc/gemmh2.hip; 22-bit significand inputs, narrower than fp32): 0 off "
                        "(the fp32-exact split-bf16 kernels, csrc/gemmx3.hip), 1 forward GEMM, "
                        "2 forward + weight gradient, 3 = 2 with the weight gradient on the "
                        "whole-row planar kernel")
    p.add_argument("--no-fused-gather", action="store_true")
    p.add_argument("--no-pipeline", action="store_true", help="sample on the training stream")
    p.add_argument("--no-hip-gemm", action="store_true", help="layer GEMMs through torch.matmul")
    p.add_argument("--early-agg", action="store_true",
                   help="aggregate-first: issue the bottom aggregation behind the sampler")
    p.add_argument("--no-priority", action="store_true", help="sampler stream at normal priority")
    p.add_argument("--sampler-high-priority", action="store_true",
                   help="sampler stream at high priority (default: high for --rng mt only)")
    p.add_argument("--training-priority", action="store_true",
                   help="the training stream at high priority, the sampler's at normal")
    p.add_argument("--model", default="gcn", choices=["gcn", "gat"],
                   help="gcn (headline) or gat (GAT_SAMPLE_ALL_GPU-style attention layers)")
    p.add_argument("--atomic-backward", action="store_true",
                   help="graph-op backward by atomic CSC scatter (no CSR transpose in the "
                        "sampler; nondeterministic sums)")
    p.add_argument("--cache-rate", type=float, default=-1.0,
                   help="feature table in pinned host memory with this fraction of the "
                        "highest-degree rows cached in HBM (GS_SAMPLE_PD_CACHE placement); "
                        "default: whole table in HBM")
    p.add_argument("--pd-cache", action="store_true",
                   help="NeutronOrch PD cache (GS_SAMPLE_PD_CACHE): per super-batch the hot "
                        "vertices' bottom layer is aggregated once and shared")
    p.add_argument("--pd-rate", type=float, default=0.2, help="PD cache: CACHE_RATE of hot vertices")
    p.add_argument("--pd-super-batch", type=int, default=4,
                   help="PD cache: batches per super-batch (PIPELINE_NUM)")
    p.add_argument("--no-fuse-act", action="store_true",
                   help="relu/dropout as torch ops instead of the GEMM epilogue")
    p.add_argument("--sampler-gate", type=int, default=0, choices=[0, 1, 2],
                   help="pipelined sampler behind the bottom forward GEMM (1), and the backward "
                        "GEMM behind the sampler (2)")
    p.add_argument("--sampler-cus", type=int, default=0,
                   help="CUs of the pipelined sampler stream: n > 0 reserved for it (training on the "
                        "rest), n < 0 the sampler confined to |n| (training on all); 0: no masks")
    p.add_argument("--no-pad-features", action="store_true",
                   help="gather from the feature table as given (no 128-byte row pitch copy)")
    p.add_argument("--no-fuse-loss", action="store_true",
                   help="output layer + loss as libtorch ops instead of the fused kernels")
    p.add_argument("--epochs", type=int, default=3,
                   help="full epochs after the timed steps; epoch time = mean of epochs 2..N")
    p.add_argument("--sampler-batches", type=int, default=32,
                   help="batches of the GPU sampler-only measurement (0: skip)")
    p.add_argument("--cpu-max-steps", type=int, default=16,
                   help="CPU baseline: at most this many batches of one epoch")
    p.add_argument("--cpu-o0-steps", type=int, default=1,
                   help="CPU baseline at the reference's -O0 build flags: batches (0: skip)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=default_cpu_threads())
    p.add_argument("--scale", type=float, default=1.0)
    p.add_argument("--train-limit", type=int, default=0,
                   help="train on the first N seeds of this rank's shard only (0: all).  PD "
                        "cache on papers100M-shaped graphs: preSample keeps every "
                        "super-batch's hot ids (~0.7 M per super-batch there)")
    p.add_argument("--secondary", action="store_true",
                   help="a secondary measurement's child run (no CPU baseline, epochs, sampler-alone "
                        "rate, interference probe or secondaries of its own)")
    p.add_argument("--no-secondary-exact", action="store_true",
                   help="skip the secondary measurement of the headline order on the f16 pair "
                        "tables (22-bit inputs) instead of the fp32-exact kernels")
    p.add_argument("--no-secondary-mt", action="store_true",
                   help="skip the secondary measurement with the reference's std::mt19937 stream "
                        "(one rank only)")
    p.add_argument("--no-secondary-af", action="store_true",
                   help="skip the secondary measurement of the reference's bottom-layer order "
                        "(aggregate-first, fp32 aggregation) beside a transform-first headline")
    p.add_argument("--rng", default="philox", choices=["philox", "mt", "mt-div"],
                   help="sampler stream: philox (per-dst counter streams, parallel) or mt: the "
                        "reference's single std::mt19937(2000) stream + uniform_int_distribution "
                        "(Lemire, libstdc++ 11; mt-div: libstdc++ <= 10), replayed bit-exactly")
    p.add_argument("--no-interference-probe", action="store_true",
                   help="skip the diagnostic training-stream-alone timing (one sampled batch "
                        "reused, no sampler beside the training stream)")
    p.add_argument("--launch-selftest", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args()


RNG_MODES = {"philox": 0, "mt": 1, "mt-div": 2}


def metric_name(args, layers) -> str:
    hops = len(layers) - 1
    model = {"gcn": "GCN" if args.weight == "sum" else "GraphSAGE", "gat": "GAT"}[args.model]
    shape = SHAPE_NAMES.get(args.shape, args.shape)
    return f"sampled-edges/sec + epoch time, {hops}-hop {model} on {shape}-shaped graph @1/2/4/8 GPUs"


def lib_sha256() -> str:
    from nts import _abi
    return hashlib.sha256(_abi.LIB_PATH.read_bytes()).hexdigest()


def main():
    args = parse()
    bad = diag_env()
    if bad:
        raise SystemExit(f"[bench] refusing to measure with diagnostic knobs set: {bad} "
                         f"(they skip work or give wrong results)")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU "
                         f"is required")
    if args.launch_selftest:
        return launch_selftest(world, rank)
    # NTS_BENCH_SHARE_GPU=1: every rank on device 0 — a rehearsal of the
    # multi-rank control flow on a one-GPU box (RCCL refuses two ranks on one
    # device, so the ranks talk over gloo: the timing collectives and the
    # gradient all-reduce, through the Communicator's host transport; the
    # numbers are not a scaling measurement)
    shared = os.environ.get("NTS_BENCH_SHARE_GPU") == "1"
    if shared:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    cdev = torch.device("cpu") if shared else dev  # device of the timing collectives
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if shared:
            dist.init_process_group("gloo")
        else:
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
    train_all = torch.nonzero(masks == 0).flatten().to(torch.int32).cpu()
    # DP: contiguous equal slices (remainder dropped so every rank runs the same
    # number of steps; the reference gives it to the last GPU,
    # toolkits/GCN_SAMPLE_ALL_MULTI.hpp:564-575)
    from nts import dist as ndist
    train = ndist.shard_nids(train_all, world, rank)
    if args.train_limit > 0:
        train = train[:args.train_limit]
    log(f"[bench] graph {args.shape}: V={V} E={En} F={F_dim} C={C}  ready in {time.time()-t0:.1f}s")
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline and not args.secondary
    src_host = g.src.cpu().numpy().view(np.uint32) if want_cpu else None
    dst_host = g.dst.cpu().numpy().view(np.uint32) if want_cpu else None
    del g

    if shared:
        comm = ndist.make_host_communicator(E, world, rank) if world > 1 else None
    else:
        comm = ndist.make_communicator(E, world, rank, local_rank)
    rccl_ranks = None  # ranks of the RCCL communicator as RCCL reports them
    if comm is not None and not comm.host_transport:
        rccl_ranks, my = comm.rccl_count()
        if rccl_ranks != world or my != rank:
            raise SystemExit(f"[bench] RCCL communicator has {rccl_ranks} ranks (this one {my}), "
                             f"expected {world} (this one {rank})")

    fan = [int(x) for x in args.fanout.split("-")]
    layers = ([int(x) for x in args.layers.split("-")] if args.layers else [F_dim, args.hidden, C])
    if layers[0] != F_dim or len(layers) != len(fan) + 1:
        raise SystemExit(f"--layers must start at the feature width {F_dim} and have one more "
                         f"entry than --fanout")
    cfg = host.gcn_config(layers, fan, args.batch, learn_rate=0.001, weight_decay=1e-4,
                          drop_rate=0.5, rng_mode=RNG_MODES[args.rng], weight=args.weight,
                          fused_gather=not args.no_fused_gather, profile=True,
                          pipeline=not args.no_pipeline, hip_gemm=not args.no_hip_gemm,
                          transform_first=args.transform_first, early_aggregate=args.early_agg,
                          sampler_priority=(-1 if args.training_priority else
                                            0 if args.no_priority else
                                            1 if args.sampler_high_priority else 2),
                          fuse_activation=not args.no_fuse_act,
                          fuse_loss=not args.no_fuse_loss, sampler_cus=args.sampler_cus,
                          sampler_gate=args.sampler_gate,
                          pad_features=not args.no_pad_features, cache_rate=args.cache_rate,
                          deterministic_backward=not args.atomic_backward,
                          gat=args.model == "gat", gemm=args.gemm, pair_table=args.pair_table, pd_cache=args.pd_cache,
                          pd_rate=args.pd_rate, pd_super_batch=args.pd_super_batch)
    log(f"[bench] building the driver (feature placement, PD-cache preSample: may take a while "
        f"on large graphs)")
    t0 = time.time()
    drv = E.GCN_SAMPLE_ALLGPU_impl(G, feat, labels, train, cfg, comm)
    log(f"[bench] driver ready in {time.time() - t0:.1f}s")
    tf = bool(drv.transform_first)

    def step():
        if not drv.sample_not_finished():
            drv.restart()
        drv.train_batch()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    def sum_over_ranks(x: float) -> float:
        if world == 1:
            return x
        import torch.distributed as dist
        t = torch.tensor([x], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t[0])

    for _ in range(args.warmup):
        step()
    drv.synchronize()
    drv.reset_stats()
    if comm is not None:  # the gradient exchange's own time per step (below)
        comm.timing_reset()
        comm.set_timing(True)

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drv.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    prof = drv.resolve_profile()
    allreduce = None
    if comm is not None:
        comm.set_timing(False)
        ar = comm.timing_stats()
        allreduce = {"us_per_step": max_over_ranks(float(ar["us_per_call"])) if ar["calls"] else None,
                     "calls": int(ar["calls"]),
                     "how": ("HIP events around the RCCL call on the stream it runs on (max over ranks)"
                             if ar["how"] == "hip-events" else
                             "host wall time of the blocking host-transport call (max over ranks)")}
    edges_local = float(drv.batch_edges)
    sample_s = float(drv.sample_time)
    train_host_s = float(drv.train_time)
    elapsed = max_over_ranks(elapsed)
    edges = sum_over_ranks(edges_local)

    # sizes of the last timed batch (before the epoch runs replace them)
    layer_sizes = [{"v": int(l["v_size"]), "src": int(l["src_size"]), "e": int(l["e_size"])}
                   for l in drv.last_layers]
    # ---- epoch time (mean of epochs 2..N) ----------------------------
    epoch_times = []
    for _ in range(0 if args.secondary else max(args.epochs, 0)):
        drv.restart()
        barrier()
        te = time.perf_counter()
        drv.run_epoch()
        drv.synchronize()
        barrier()
        epoch_times.append(max_over_ranks(time.perf_counter() - te))
    drv.resolve_profile()
    n_train_per_gpu = int(train.numel())
    batches_per_epoch = -(-n_train_per_gpu // args.batch)
    if len(epoch_times) >= 2:
        epoch_s, epoch_kind = float(np.mean(epoch_times[1:])), (
            f"measured: mean of epochs 2..{len(epoch_times)} over this rank's training shard")
    elif epoch_times:
        epoch_s, epoch_kind = epoch_times[0], "measured: one epoch (the first)"
    else:
        epoch_s, epoch_kind = elapsed / args.steps * batches_per_epoch, "ms_per_step x batches/epoch"

    # ---- diagnostic: the training stream without the sampler beside it -----------
    alone = None
    if (args.model == "gcn" and not args.no_interference_probe and args.steps > 0
            and not args.secondary
            and not args.no_pipeline):
        drv.set_diag_reuse_sample(True)
        for _ in range(args.warmup):
            step()
        drv.synchronize()
        drv.reset_stats()
        barrier()
        ta = time.perf_counter()
        for _ in range(args.steps):
            step()
        drv.synchronize()
        barrier()
        el_alone = max_over_ranks(time.perf_counter() - ta)
        prof_alone = drv.resolve_profile()
        drv.set_diag_reuse_sample(False)
        alone = {"ms_per_step": el_alone / args.steps * 1e3, "steps": args.steps,
                 "interference_ms_per_step": (elapsed - el_alone) / args.steps * 1e3,
                 "kernel_avg_us": {k: {"alone": round(v["ms"] / v["calls"] * 1e3, 1),
                                       "pipelined": round(prof[k]["ms"] / prof[k]["calls"] * 1e3, 1)}
                                   for k, v in prof_alone.items()
                                   if v["calls"] and k in prof and prof[k]["calls"]},
                 "note": "diagnostic, not a throughput: one sampled batch reused every step, "
                         "so the training stream runs without the pipelined sampler beside it"}

    # ---- GPU sampler alone (SURVEY §8d sampler-only rate) -------------------------
    sampler_only = None
    if args.sampler_batches > 0 and args.model == "gcn" and not args.secondary:
        L = len(fan)
        csr = [not args.atomic_backward] * (L - 1) + [tf]
        wt = {"sum": E.WeightType.Sum, "mean": E.WeightType.Mean,
              "mean-sampled": E.WeightType.MeanSampled}[args.weight]
        r = E.sampler_throughput(G, train, args.batch, fan, wt, RNG_MODES[args.rng],
                                 args.sampler_batches, csr)
        sampler_only = {"value": sum_over_ranks(r["edges"]) / max_over_ranks(r["seconds"]),
                        "unit": "sampled-edges/s", "batches_per_gpu": int(r["batches"]),
                        "note": "GPU sampler alone on its stream (3 batches in flight), all ranks"}

    # ---- secondary orders / arithmetic on the same workload ----------------------
    # Each secondary runs as a fresh CHILD process (`bench.py ... --secondary`,
    # one rank, nothing else on the GPU: this process is idle and holds no
    # stream of its own in flight), so that no driver, stream or sampler of
    # the headline run sits beside it (measured in round 4: the MT secondary
    # read 5.1 ms/step beside them against 3.9 alone).
    def child_secondary(overrides: dict, note: str):
        # the parent's own workload flags (every flag the headline
        # was run with, --rng / --no-pad-features / --cache-rate ... included)
        cmd = [sys.executable, str(ROOT / "bench.py"), *child_argv(sys.argv[1:], overrides)]
        log(f"[bench] secondary ({note}): {' '.join(cmd[2:])}")
        t0 = time.time()
        r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, env=dict(os.environ))
        line = None
        for out in r.stdout.splitlines():
            try:
                obj = json.loads(out)
            except ValueError:
                continue
            if isinstance(obj, dict) and "metric" in obj:
                line = obj
        if r.returncode != 0 or line is None:
            return {"error": f"child exited {r.returncode}", "argv": " ".join(cmd[2:])}
        rl = line.get("roofline") or {}
        return {"value": line["value"], "unit": line["unit"], "ms_per_step": line["ms_per_step"],
                "steps": line["steps"], "warmup": line["warmup"], "dtype": line["dtype"],
                "bottom_layer": line["config"].get("bottom_layer"),
                "roofline": {k: rl.get(k) for k in ("kernel", "bound", "achieved", "peak", "unit",
                                                      "frac", "avg_launch_ms")},
                "argv": " ".join(cmd[2:]), "child_wall_s": round(time.time() - t0, 1),
                "measured": "fresh child process, the headline run idle"}

    secondary = None  # the reference's bottom-layer order
    pair_tf = None    # the headline order on the f16 pair tables (22-bit inputs)
    mt_ref = None     # the reference's generator stream
    if (tf and args.model == "gcn" and args.steps > 0 and world == 1 and not args.secondary):
        if not args.no_secondary_af:
            secondary = {
                "bottom_layer": "aggregate-first (A X) W, the reference's order: fp32 aggregation "
                                "bit-exact vs MiniBatchFuseOp, split-bf16 GEMMs (fp32-accurate)",
                **child_secondary({"--transform-first": 0, "--pair-table": 0},
                                  "the reference's bottom-layer order")}
        if args.pair_table == 0 and not args.no_secondary_exact:
            pair_tf = {
                "bottom_layer": "transform-first A (X W) with the bottom-layer GEMMs on the feature "
                                "table's f16 pair tables: 22-bit significand inputs (NARROWER than "
                                "fp32), 3 f16 MFMA products, fp32 accumulate",
                **child_secondary({"--transform-first": 1, "--pair-table": 3},
                                  "f16 pair tables")}
    # the same workload on the reference's own generator stream (std::mt19937
    # + Lemire, every sampled array bit-exact vs the reference's serial order)
    if (args.model == "gcn" and args.rng == "philox" and world == 1 and args.steps > 0
            and not args.no_secondary_mt and not args.secondary):
        mt_ref = {
            "rng": "std::mt19937(2000) + Lemire, the reference's stream (FastSampler::sample_fast)",
            **child_secondary({"--rng": "mt"},
                              "the reference's MT19937 stream")}

    value = edges / elapsed
    rl = roofline(prof, args, layers, world)
    result = {
        "metric": metric_name(args, layers),
        "value": value,
        "unit": "sampled-edges/s",
        "n_gpus": world,
        "rccl_ranks": rccl_ranks,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype_name(args, tf),
        "data": "synthetic Chung-Lu power-law graph (seed 2024), N(0,1) fp32 features (seed 7), uniform labels",
        "config": {
            "workload": workload_name(args, layers, V, En, tf),
            "global_batch": args.batch * world,
            "parallelism": f"dp{world}" + ("-shared-gpu-rehearsal (gloo all-reduce through host copies)" if shared and world > 1 else ""),
            "gradient_exchange": ("none (one rank)" if comm is None else
                                  "gloo host transport" if comm.host_transport else
                                  f"RCCL all-reduce, {rccl_ranks} ranks"),
            "allreduce_us_per_step": allreduce["us_per_step"] if allreduce else None,
            "allreduce_timing": allreduce,
            "training_stream_alone": alone,
            "fanout": args.fanout,
            "epoch_time_s": epoch_s,
            "epoch_time_kind": epoch_kind,
            "epoch_times_s": epoch_times,
            "batches_per_epoch_per_gpu": batches_per_epoch,
            "train_seeds_per_gpu": int(train.numel()),
            "gpu_sampler_only": sampler_only,
            "host_sampler_wait_s_per_step": sample_s / args.steps,
            "host_train_issue_s_per_step": train_host_s / args.steps,
            "bottom_layer": "transform-first A(X W)" if tf else "aggregate-first (A X) W",
            "gemm": {"f32": "fp32-input MFMA",
                     "split3": "fp32 split into 3 bf16 pieces, 6 products, fp32 accumulate"}[args.gemm]
                    + ("; bottom layer: the feature table's f16 pair tables (two f16 pieces + "
                       "power-of-two row scale, 3 f16 MFMA products, fp32 accumulate)"
                       if tf and args.pair_table >= 1 else ""),
            "layer_sizes_top_down": layer_sizes,
            "reference_order_secondary": secondary,
            "pair_table_secondary": pair_tf,
            "reference_stream_secondary": mt_ref,
            "profile_meta": {"argv": " ".join(sys.argv[1:]), "lib_sha256": lib_sha256(),
                             "nts_env": nts_env(),
                             "workload": pmc_workload(args, layers, world)},
        },
        "roofline": rl,
    }
    if want_cpu:
        result["cpu_baseline"] = cpu_baseline(args, G, feat, labels, train, fan, layers, V)
        if sampler_only is not None and result["cpu_baseline"].get("sampler_only"):
            result["config"]["gpu_vs_cpu_sampler_only"] = (
                sampler_only["value"] / result["cpu_baseline"]["sampler_only"]["value"])
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def dtype_name(args, tf) -> str:
    if tf and args.pair_table >= 1:
        return ("f16-pair (bottom-layer GEMMs on the feature table's f16 pair tables: 22-bit "
                "significand inputs, narrower than fp32; 3 f16 MFMA products, fp32 accumulate)")
    if args.gemm == "split3":
        return ("fp32 (GEMM inputs fp32, split exactly into three bf16 pieces in the kernels, "
                "6 bf16 MFMA products, fp32 accumulate; aggregation fp32)")
    return "fp32"


def workload_name(args, layers, V, En, tf) -> str:
    if args.model == "gat":
        kind, model = "GAT_SAMPLE_ALL_GPU", "GAT"
    else:
        kind = ("GS" if args.weight != "sum" else "GCN") + "_SAMPLE_ALLGPU"
        model = {"sum": "GCN", "mean": "GraphSAGE (mean, CPU formula)",
                 "mean-sampled": "GraphSAGE (mean by sampled count, GPU kernel formula)"}[args.weight]
    s = (f"{kind}-style {len(layers) - 1}-layer {model} {'-'.join(map(str, layers))}, fanout "
         f"{args.fanout}, batch {args.batch}/GPU, {args.shape}-shaped synthetic (V={V}, E={En}); "
         f"GPU sampler ({RNG_NAMES[args.rng]}{', pipelined' if not args.no_pipeline else ''}) + "
         + (("transform-first bottom layer (row-gathered "
             + ("f16 pair-table" if args.pair_table >= 1 else "MFMA")
             + " GEMMs, aggregation + relu/dropout)") if tf else "fused gather/aggregation")
         + " + " + ("torch" if args.no_hip_gemm else
                    {"f32": "fp32-input MFMA", "split3": "fp32-accurate split-bf16 MFMA"}[args.gemm])
         + " GEMMs + fused loss + fused Adam")
    if args.cache_rate >= 0:
        s += (f"; features in pinned host memory, {args.cache_rate:.0%} of rows (highest degree) "
              f"cached in HBM")
    if args.pd_cache:
        s += (f"; NeutronOrch PD cache (GS_SAMPLE_PD_CACHE): {args.pd_rate:.0%} hot vertices per "
              f"super-batch of {args.pd_super_batch} batches, their bottom layer shared")
    return s


RNG_NAMES = {"philox": "Philox", "mt": "MT19937 reference stream, Lemire",
             "mt-div": "MT19937 reference stream, DIV"}


def roofline(prof: dict, args, layers, world) -> dict:
    """Dominant kernel by device time over the timed steps (HIP events on the
    stream that launches it), its algorithmic units / average launch time vs
    the MI355X peak; every profiled kernel listed under `kernels`."""
    kernels = {}
    F, N = layers[0], layers[1]
    Kp = (F + 31) // 32 * 32
    for name, st in prof.items():
        if not st["calls"]:
            continue
        avg_s = st["ms"] / st["calls"] * 1e-3
        gemm = name.startswith("gather_gemm")
        per = st["units"] / st["calls"]
        pair = gemm and (args.pair_table >= (1 if name == "gather_gemm" else 2))
        if pair:
            # f16 pair-table GEMM (csrc/gemmh2.hip): three f16 MFMA products per
            # fp32 product, against the dense f16 peak; and its algorithmic
            # bytes (each gathered pair-table row once, the fp32 B rows / output
            # rows once, W once) against HBM — the binding roof is reported
            rows = per / (2.0 * F * N)
            byt = rows * (4.0 * Kp + 4.0 * N) + 4.0 * Kp * N
            mf = 3.0 * per / avg_s / 1e12
            hb = byt / avg_s / 1e9
            k_m = {"bound": "mfma", "unit": "TFLOP/s", "achieved": mf, "peak": F16_MFMA_PEAK_TF,
                   "frac": mf / F16_MFMA_PEAK_TF}
            k_h = {"bound": "hbm", "unit": "GB/s", "achieved": hb, "peak": HBM_PEAK_GBS,
                   "frac": hb / HBM_PEAK_GBS}
            k = dict(max(k_m, k_h, key=lambda d: d["frac"]))
            k.update({"avg_launch_ms": avg_s * 1e3, "flops_per_launch": per,
                      "f16_mfma_flops_per_launch": 3.0 * per, "algorithmic_bytes_per_launch": byt,
                      "mfma_frac": k_m["frac"], "hbm_frac": k_h["frac"],
                      "arithmetic": "f16 pair table (3 f16 MFMAs per fp32 product)",
                      "calls": st["calls"], "share_of_timed_ms": st["ms"]})
            kernels[name] = k
            continue
        if gemm and args.gemm == "split3" and not args.no_hip_gemm:
            # fp32-exact row-gathered GEMM (csrc/gemmx3.hip): six bf16 MFMA
            # products per fp32 product against the dense bf16 peak; and its
            # algorithmic bytes (each gathered fp32 row of Kp floats once, the
            # other operand's / the output's rows once, W once) against HBM —
            # the binding roof is reported
            rows = per / (2.0 * F * N)
            byt = rows * (4.0 * Kp + 4.0 * N) + 4.0 * Kp * N
            mf = 6.0 * per / avg_s / 1e12
            hb = byt / avg_s / 1e9
            k_m = {"bound": "mfma", "unit": "TFLOP/s", "achieved": mf, "peak": F16_MFMA_PEAK_TF,
                   "frac": mf / F16_MFMA_PEAK_TF}
            k_h = {"bound": "hbm", "unit": "GB/s", "achieved": hb, "peak": HBM_PEAK_GBS,
                   "frac": hb / HBM_PEAK_GBS}
            k = dict(max(k_m, k_h, key=lambda d: d["frac"]))
            k.update({"avg_launch_ms": avg_s * 1e3, "flops_per_launch": per,
                      "bf16_mfma_flops_per_launch": 6.0 * per, "algorithmic_bytes_per_launch": byt,
                      "mfma_frac": k_m["frac"], "hbm_frac": k_h["frac"],
                      "arithmetic": "fp32 split into 3 bf16 pieces (6 bf16 MFMAs per fp32 product)",
                      "calls": st["calls"], "share_of_timed_ms": st["ms"]})
            kernels[name] = k
            continue
        ach = per / avg_s / (1e12 if gemm else 1e9)
        peak = FP32_MFMA_PEAK_TF if gemm else HBM_PEAK_GBS
        kernels[name] = {
            "bound": "mfma" if gemm else "hbm", "unit": "TFLOP/s" if gemm else "GB/s",
            "achieved": ach, "peak": peak, "frac": ach / peak, "avg_launch_ms": avg_s * 1e3,
            ("flops_per_launch" if gemm else "algorithmic_bytes_per_launch"): per,
            "calls": st["calls"], "share_of_timed_ms": st["ms"]}
    if not kernels:
        return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": None, "traffic": None}
    dom = max(kernels, key=lambda k: kernels[k]["share_of_timed_ms"])
    k = kernels[dom]
    rl = {"bound": k["bound"], "kernel": dom, "achieved": k["achieved"], "peak": k["peak"],
          "unit": k["unit"], "frac": k["frac"], "traffic": None,
          "avg_launch_ms": k["avg_launch_ms"], "kernels": kernels,
          "timing": ("HIP events on the launching stream over the timed steps, one kernel "
                     "class per step in rotation (KernelProfiler, nts_host.hpp)")}
    attach_pmc(rl, dom, args, layers, world)
    return rl


def pmc_workload(args, layers, world) -> str:
    return (f"{args.shape}/{args.batch}/{args.fanout}/{'-'.join(map(str, layers))}/{args.weight}/"
            f"w{world}/tf{args.transform_first}/{args.model}/c{args.cache_rate}/{args.gemm}"
            + (f"/pd{args.pd_rate}x{args.pd_super_batch}" if args.pd_cache else "")
            + (f"/rng-{args.rng}" if args.rng != "philox" else ""))


def attach_pmc(rl, dom, args, layers, world):
    """HBM bytes per launch from a committed rocprofv3 --pmc pass
    (profiles/pmc_*.json) — only if it was taken on this exact libnts_hip.so
    build, this kernel and this workload; otherwise traffic stays null and
    the reason is stated."""
    wl = pmc_workload(args, layers, world)
    sha = lib_sha256()
    why = "no PMC pass recorded for this build/kernel/workload"
    for f in sorted((ROOT / "profiles").glob("pmc_*.json"), reverse=True):
        try:
            info = json.loads(f.read_text())
        except Exception:
            continue
        # (the pass's own dominant kernel may differ from this run's when two
        # kernels are close: any kernel of the pass that maps to `dom` counts)
        if info.get("workload") != wl:
            continue
        if info.get("lib_sha256") != sha:
            why = f"{f.name} was taken on another libnts_hip.so build: not attached"
            continue
        for kname, kv in info.get("kernels", {}).items():
            if kv.get("profiler_kernel") == dom and kv.get("hbm_bytes_per_launch"):
                tb = float(kv["hbm_bytes_per_launch"])
                rl["traffic"] = tb
                rl["traffic_source"] = f"{f.name} ({kname})"
                rl["traffic_GBs"] = tb / (rl["avg_launch_ms"] * 1e-3) / 1e9
                rl["traffic_frac_of_hbm_peak"] = rl["traffic_GBs"] / HBM_PEAK_GBS
                return
    rl["traffic_note"] = why


def cpu_info() -> dict:
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {**cpu_share(), "cpu_model": model}


def cpu_baseline(args, G, feat, labels, train, fan, layers, V):
    """The reference CPU path restated (oracle/ref_cpu.cpp; toolkits/GCN_CPU_SAMPLE.hpp:194-256)
    timed on this host over one epoch of the same workload (at most
    --cpu-max-steps batches): sample_fast (OpenMP, thread-local mt19937),
    get_feature, MiniBatchFuseOp fwd/bwd (CAS backward), libtorch CPU GEMM and
    learnC2C_with_decay_Adam (core/NtsScheduler.hpp:863-880)."""
    from oracle import oracle as orc
    threads = max(1, args.cpu_threads)
    torch.set_num_threads(threads)
    col = G.column_offset.cpu().numpy().view(np.uint64)
    rows = G.row_indices.cpu().numpy().view(np.uint32)
    in_d = G.in_degree.cpu().numpy().view(np.uint32)
    out_d = G.out_degree.cpu().numpy().view(np.uint32)
    feat_h = feat.cpu().numpy()
    lab_h = labels.cpu()
    ids = train.numpy().astype(np.uint32)
    n_batches = -(-ids.size // args.batch)
    L = len(fan)
    wmean = args.weight != "sum"
    wt = {"sum": orc.W_SUM, "mean": orc.W_MEAN, "mean-sampled": orc.W_MEAN_SAMPLED}[args.weight]

    def run(steps, variant):
        with orc.variant(variant):
            s = orc.Sampler(col, rows, in_d, out_d, fan, seed=2000, rng_mode=orc.RNG_MT_LEMIRE,
                            order_mode=orc.ORDER_UNORDERED_MAP)
            gen = torch.Generator().manual_seed(0)
            W = [torch.empty(a, b).uniform_(-(6 / (a + b)) ** 0.5, (6 / (a + b)) ** 0.5,
                                            generator=gen).requires_grad_()
                 for a, b in zip(layers[:-1], layers[1:])]
            M = [torch.zeros_like(w) for w in W]
            Vv = [torch.zeros_like(w) for w in W]
            b1, b2, lr, wd, eps = 0.9, 0.999, 0.001, 1e-4, 1e-9
            b1t, b2t = b1, b2  # Parameter::beta1_t/beta2_t, advanced by next()
            edges, t_all, t_samp = 0, 0.0, 0.0
            for it in range(steps):
                seeds = ids[it * args.batch:(it + 1) * args.batch]
                t0 = time.perf_counter()
                ls = s.sample(seeds, it, wt, True, threads)
                t1 = time.perf_counter()
                # GCN_CPU_SAMPLE forward: hop = L-1-l, features of the outermost source
                X = torch.from_numpy(orc.get_feature(ls[-1]["source"], feat_h, threads))
                Ys = []
                for l in range(L):
                    lay = ls[L - 1 - l]
                    Y = torch.from_numpy(orc.fuse_fwd(lay, X.detach().numpy(), out_d, in_d,
                                                      weight_mean=wmean, threads=threads))
                    if l > 0:
                        Y.requires_grad_()
                    Ys.append((Y, X))
                    Z = Y @ W[l]
                    X = torch.dropout(torch.relu(Z), 0.5, True) if l < L - 1 else Z
                tgt = lab_h[torch.from_numpy(ls[0]["destination"].astype(np.int64))]
                loss = torch.nn.functional.nll_loss(X.log_softmax(1), tgt)
                loss.backward()
                for l in range(L - 1, 0, -1):  # graph-op backward (not the bottom one)
                    Y, Xin = Ys[l]
                    gX = orc.fuse_bwd(ls[L - 1 - l], Y.grad.numpy(), out_d, in_d,
                                      weight_mean=wmean, threads=threads)
                    Xin.backward(torch.from_numpy(gX))
                with torch.no_grad():  # learnC2C_with_decay_Adam, bias-corrected
                    for i, w in enumerate(W):
                        wg = w.grad + wd * w
                        M[i] = b1 * M[i] + (1 - b1) * wg
                        Vv[i] = b2 * Vv[i] + (1 - b2) * wg * wg
                        w -= lr * (M[i] / (1 - b1t)) / (torch.sqrt(Vv[i] / (1 - b2t)) + eps)
                        w.grad = None
                    b1t, b2t = b1t * b1, b2t * b2
                t2 = time.perf_counter()
                t_samp += t1 - t0
                t_all += t2 - t0
                edges += sum(l["e_size"] for l in ls)
            return edges, t_all, t_samp

    steps = max(1, min(args.cpu_max_steps, n_batches))
    edges, t_all, t_samp = run(steps, "O3")
    out = {
        "value": edges / t_all,
        "unit": "sampled-edges/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{steps} of the {n_batches} GCN_CPU_SAMPLE training steps of one epoch, batch "
                   f"{args.batch}, same graph ({edges} sampled edges, {t_all:.1f}s), OpenMP "
                   f"{threads} threads, oracle/ref_cpu.cpp -O3 x86-64-v3 + torch CPU"),
        "sampler_only": {"value": edges / t_samp, "unit": "sampled-edges/s",
                         "note": "sample_fast alone (OpenMP, thread-local mt19937)"},
        "epoch_time_s": t_all / steps * n_batches,
        "epoch_time_kind": ("measured: one full epoch" if steps == n_batches
                            else f"estimate: per-step time of {steps} steps x {n_batches} batches"),
        "threads_rule": ("min(nproc - 1 (the reference's default, core/FullyRepGraph.hpp:49), "
                         "affinity_cpus, cpu_quota (cgroup CFS), omp_num_threads (the job's "
                         "declared CPU share)); --cpu-threads overrides"),
        **cpu_info(),
    }
    if args.cpu_o0_steps > 0:
        e0, t0_all, t0_s = run(min(args.cpu_o0_steps, n_batches), "O0")
        out["O0_build"] = {"value": e0 / t0_all, "sampler_only": e0 / t0_s,
                           "unit": "sampled-edges/s",
                           "note": (f"{min(args.cpu_o0_steps, n_batches)} step(s) with ref_cpu.cpp "
                                    f"built -O0 like the reference's shipped build "
                                    f"(CMakeLists.txt:109); torch CPU ops unchanged")}
    return out


if __name__ == "__main__":
    main()
