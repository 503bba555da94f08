"""The N>1 data-parallel path on CPU: world_size 2 over gloo.

Checks the pieces the GPU ranks use — equal seed shards, the RCCL unique-id
broadcast through torch.distributed, and the fused SUM all-reduce of the layer
gradients — with the CPU oracle computing each rank's gradients.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as orc
from nts import dist as ndist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _graph():
    rng = np.random.default_rng(0)
    V, E = 800, 12000
    src = rng.integers(0, V, E).astype(np.uint32)
    dst = rng.integers(0, V, E).astype(np.uint32)
    src = np.concatenate([src, dst, np.arange(V, dtype=np.uint32)])
    dst = np.concatenate([dst, src[:E], np.arange(V, dtype=np.uint32)])
    col, rows = orc.build_csc(V, src, dst)
    od, idg = orc.degrees(V, src, dst)
    feat = rng.standard_normal((V, 16)).astype(np.float32)
    labels = torch.from_numpy(rng.integers(0, 4, V))
    return V, col, rows, od, idg, feat, labels


def _local_grads(seeds, W0, W1):
    V, col, rows, od, idg, feat, labels = _graph()
    s = orc.Sampler(col, rows, idg, od, [5, 3], rng_mode=orc.RNG_PHILOX, order_mode=orc.ORDER_DRAW)
    l0, l1 = s.sample(seeds.astype(np.uint32), 0)
    W = [torch.from_numpy(W0).requires_grad_(), torch.from_numpy(W1).requires_grad_()]
    X0 = orc.get_feature(l1["source"], feat)
    Y0 = torch.from_numpy(orc.fuse_fwd(l1, X0, od, idg))
    X1 = torch.relu(Y0 @ W[0])
    Y1 = torch.from_numpy(orc.fuse_fwd(l0, X1.detach().numpy(), od, idg)).requires_grad_()
    X2 = (Y1 @ W[1]).log_softmax(1)
    tgt = labels[torch.from_numpy(l0["destination"].astype(np.int64))]
    torch.nn.functional.nll_loss(X2, tgt).backward()
    gX1 = orc.fuse_bwd(l0, Y1.grad.numpy(), od, idg)
    X1.backward(torch.from_numpy(gX1))
    return [w.grad.numpy().copy() for w in W]


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        train = np.random.default_rng(3).permutation(601).astype(np.uint32)  # 601: odd remainder
        shard = ndist.shard_nids(train, world, rank)
        n_steps = torch.tensor([ndist.steps_per_epoch(len(shard), 64)])
        dist.all_reduce(n_steps, op=dist.ReduceOp.MAX)
        uid = ndist.broadcast_unique_id(lambda: os.urandom(128), rank)
        rng = np.random.default_rng(9)
        W0 = (rng.standard_normal((16, 8)) * 0.3).astype(np.float32)
        W1 = (rng.standard_normal((8, 4)) * 0.3).astype(np.float32)
        grads = _local_grads(shard[:64], W0, W1)

        def allreduce(buf):
            t = torch.from_numpy(buf)
            dist.all_reduce(t, op=dist.ReduceOp.SUM)

        summed = ndist.global_grad_sum(grads, allreduce)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), uid=np.frombuffer(uid, np.uint8),
                 g0=summed[0], g1=summed[1], n_local=len(shard), steps=int(n_steps))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_data_parallel(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{i}.npz") for i in range(world)]
    assert np.array_equal(r[0]["uid"], r[1]["uid"])                # same RCCL id on every rank
    assert int(r[0]["n_local"]) == int(r[1]["n_local"]) == 300      # equal shards, remainder dropped
    assert int(r[0]["steps"]) == int(r[1]["steps"])
    for k in ("g0", "g1"):
        assert np.array_equal(r[0][k], r[1][k])                     # identical update on both ranks
    # == the sum of the per-rank gradients computed in one process
    train = np.random.default_rng(3).permutation(601).astype(np.uint32)
    rng = np.random.default_rng(9)
    W0 = (rng.standard_normal((16, 8)) * 0.3).astype(np.float32)
    W1 = (rng.standard_normal((8, 4)) * 0.3).astype(np.float32)
    ref = [np.zeros_like(W0), np.zeros_like(W1)]
    for rank in range(world):
        g = _local_grads(ndist.shard_nids(train, world, rank)[:64], W0, W1)
        ref = [a + b for a, b in zip(ref, g)]
    np.testing.assert_allclose(r[0]["g0"], ref[0], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(r[0]["g1"], ref[1], rtol=1e-6, atol=1e-7)


def test_shard_nids_equal_and_disjoint():
    ids = np.arange(1003)
    parts = [ndist.shard_nids(ids, 4, r) for r in range(4)]
    assert all(len(p) == 250 for p in parts)
    assert len(np.unique(np.concatenate(parts))) == 1000
    with pytest.raises(ValueError):
        ndist.shard_nids(ids, 2, 2)
