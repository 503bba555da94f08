"""The C++ data-parallel path executed with two ranks that actually sum
(GCN_SAMPLE_ALL_MULTI::Update, /root/reference/toolkits/GCN_SAMPLE_ALL_MULTI.hpp:367-377,
seed split :564-587): each rank's GCN_SAMPLE_ALLGPU_impl trains its own equal
shard and every step all-reduces (SUM) the fused gradient bucket through its
Communicator before Adam; the initial weights are broadcast from rank 0.

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


def _setup(world, rank, comm, tf):
    from nts import dist as ndist, host, synthetic
    E = host.ext()
    dev = torch.device("cuda:0")
    g = synthetic.chung_lu(6000, 180000, 20.0, device=dev, seed=3)
    G = E.FullyRepGraph.from_edges(g.src, g.dst, g.n_vertices)
    feat = synthetic.features(g.n_vertices, 64, device=dev)
    labels, masks = synthetic.labels_masks(g.n_vertices, 7, device=dev)
    train = torch.nonzero(masks == 0).flatten().to(torch.int32).cpu()
    shard = ndist.shard_nids(train, world, rank)
    cfg = host.gcn_config([64, 128 if tf else 32, 7], [10, 5], 128, learn_rate=0.01, drop_rate=0.5,
                          shuffle=False, transform_first=tf)
    if comm is None:
        return E.GCN_SAMPLE_ALLGPU_impl(G, feat, labels, shard, cfg)
    return E.GCN_SAMPLE_ALLGPU_impl(G, feat, labels, shard, cfg, comm)


def _train(drv):
    for _ in range(STEPS):
        if not drv.sample_not_finished():
            drv.restart()
        drv.train_batch()
    drv.synchronize()
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
