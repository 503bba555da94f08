"""The C++ data-parallel path executed with two ranks that actually sum
(GCN_SAMPLE_ALL_MULTI::Update, /root/reference/toolkits/GCN_SAMPLE_ALL_MULTI.hpp:367-377,
seed split :564-587): each rank's GCN_SAMPLE_ALLGPU_impl trains its own equal
shard and every step all-reduces (SUM) the fused gradient bucket through its
Communicator before Adam; the initial weights are broadcast from rank 0.

The overlap path (the all-reduce on its own stream, the Adam step deferred
until the next batch first reads W; on by default at > 1 rank) and the
in-order path (overlap_allreduce=0) must end bit-identical, and every rank
must run the same number of steps across an epoch boundary.

Both ranks share the one GPU, so the Communicator runs its host transport
(RCCL refuses two ranks on one device): torch.distributed over gloo in two
processes, and — as the reference itself runs it, one thread per device in
one process — two threads summing in a fixed order.  Checked: both ranks end
with bit-identical weights, the two transports agree bit for bit, and the sum
is real (the result differs from either shard trained alone).
"""
import os
import socket
import threading

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
STEPS = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(world, rank, comm, tf, overlap=-1, batch=128):
    from nts import dist as ndist, host, synthetic
    E = host.ext()
    dev = torch.device("cuda:0")
    g = synthetic.chung_lu(6000, 180000, 20.0, device=dev, seed=3)
    G = E.FullyRepGraph.from_edges(g.src, g.dst, g.n_vertices)
    feat = synthetic.features(g.n_vertices, 64, device=dev)
    labels, masks = synthetic.labels_masks(g.n_vertices, 7, device=dev)
    train = torch.nonzero(masks == 0).flatten().to(torch.int32).cpu()
    shard = ndist.shard_nids(train, world, rank)
    cfg = host.gcn_config([64, 128 if tf else 32, 7], [10, 5], batch, learn_rate=0.01, drop_rate=0.5,
                          shuffle=False, transform_first=tf, overlap_allreduce=overlap)
    if comm is None:
        return E.GCN_SAMPLE_ALLGPU_impl(G, feat, labels, shard, cfg)
    return E.GCN_SAMPLE_ALLGPU_impl(G, feat, labels, shard, cfg, comm)


def _train(drv, steps=STEPS):
    restarts = 0
    for _ in range(steps):
        if not drv.sample_not_finished():
            drv.restart()
            restarts += 1
        drv.train_batch()
    drv.synchronize()
    if steps != STEPS:
        return [w.cpu() for w in drv.weights()], int(drv.batches), restarts
    return [w.cpu() for w in drv.weights()]


def _gloo_worker(rank, world, port, out_dir, tf):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nts import dist as ndist, host
        torch.cuda.set_device(0)
        comm = ndist.make_host_communicator(host.ext(), world, rank)
        w = _train(_setup(world, rank, comm, tf))
        torch.save(w, os.path.join(out_dir, f"w{rank}.pt"))
    finally:
        dist.destroy_process_group()


class _ThreadPair:
    """Two ranks as two threads of one process: rank 0 sums rank 0's buffer +
    rank 1's (the order gloo's two-rank sum is bit-identical to)."""

    def __init__(self):
        self.bar = threading.Barrier(2)
        self.bufs = [None, None]
        self.res = None

    def collective(self, rank):
        def f(t, op, root):
            self.bufs[rank] = t
            self.bar.wait()
            if rank == 0:
                self.res = (self.bufs[0] + self.bufs[1]) if op == 0 else self.bufs[root].clone()
                torch.cuda.synchronize()
            self.bar.wait()
            t.copy_(self.res)
            torch.cuda.synchronize()
            self.bar.wait()
        return f


@pytest.mark.parametrize("tf", [0, 1])
def test_two_ranks_sum_gradients_through_the_cpp_driver(tmp_path, tf):
    world = 2
    mp.spawn(_gloo_worker, args=(world, _free_port(), str(tmp_path), tf), nprocs=world, join=True)
    gw = [torch.load(tmp_path / f"w{r}.pt", weights_only=True) for r in range(world)]
    for a, b in zip(gw[0], gw[1]):
        assert torch.equal(a, b), "ranks diverged"
    # the same two ranks as two threads of one process
    from nts import dist as ndist, host
    E = host.ext()
    pair = _ThreadPair()
    out = [None, None]
    err = []

    def run(rank):
        try:
            comm = ndist.make_host_communicator(E, world, rank, pair.collective(rank))
            out[rank] = _train(_setup(world, rank, comm, tf))
        except Exception as e:  # surfaced below
            err.append(e)
            pair.bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not err, err
    for a, b, c in zip(out[0], out[1], gw[0]):
        assert torch.equal(a, b) and torch.equal(a, c), "thread transport != gloo transport"
    # the all-reduce is real: training on rank 0's shard alone ends elsewhere
    alone = _train(_setup(world, 0, None, tf))
    assert not all(torch.equal(a, b) for a, b in zip(alone, gw[0]))


def _epoch_worker(rank, world, port, out_dir, overlap):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nts import dist as ndist, host
        torch.cuda.set_device(0)
        comm = ndist.make_host_communicator(host.ext(), world, rank)
        # 1,950 seeds per rank at batch 512: 4 steps per epoch, 7 steps cross one boundary
        w, steps, restarts = _train(_setup(world, rank, comm, 1, overlap=overlap, batch=512), 7)
        torch.save({"w": w, "steps": steps, "restarts": restarts},
                   os.path.join(out_dir, f"e{overlap}_{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_overlapped_allreduce_matches_in_order_update_across_an_epoch(tmp_path):
    """overlap_allreduce=1 (deferred Adam behind the all-reduce on its own
    stream) == overlap_allreduce=0 (all-reduce then Adam in order), bit for
    bit, with both ranks at the same step count through an epoch boundary."""
    world = 2
    res = {}
    for overlap in (0, 1):
        mp.spawn(_epoch_worker, args=(world, _free_port(), str(tmp_path), overlap), nprocs=world,
                 join=True)
        res[overlap] = [torch.load(tmp_path / f"e{overlap}_{r}.pt", weights_only=True)
                        for r in range(world)]
    for overlap in (0, 1):
        r0, r1 = res[overlap]
        assert r0["steps"] == r1["steps"] == 7 and r0["restarts"] == r1["restarts"] == 1
        for a, b in zip(r0["w"], r1["w"]):
            assert torch.equal(a, b), f"ranks diverged (overlap={overlap})"
    for a, b in zip(res[0][0]["w"], res[1][0]["w"]):
        assert torch.equal(a, b), "deferred optimizer step != in-order step"


def test_bench_gpus_2_launches_two_ranks_on_one_gpu():
    """`bench.py --gpus 2` with no launcher on a one-GPU box: the parent starts
    torch.distributed.run as a child, both ranks train on device 0 (the
    shared-GPU rehearsal, gloo host transport), and the relayed line says 2."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK") and not k.startswith("NTS_")}
    env["NTS_BENCH_SHARE_GPU"] = "1"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--shape", "tiny",
                        "--batch", "128", "--steps", "3", "--warmup", "1", "--epochs", "0",
                        "--sampler-batches", "0", "--no-cpu-baseline", "--no-secondary-af"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["rccl_ranks"] is None
    assert line["config"]["gradient_exchange"] == "gloo host transport"
    assert line["config"]["allreduce_us_per_step"] > 0
    assert line["config"]["allreduce_timing"]["calls"] == 3
    assert line["config"]["global_batch"] == 256 and line["value"] > 0
