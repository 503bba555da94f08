"""Data-parallel plumbing (one process per GPU).

Replaces the reference's single-process multi-GPU setup of
GCN_SAMPLE_ALL_MULTI (toolkits/GCN_SAMPLE_ALL_MULTI.hpp:89-113, 564-587):
  * seeds: contiguous split of the (shuffled) training ids into `world`
    slices; the reference hands the remainder to the last GPU, which gives the
    ranks different step counts (a collective deadlock risk) — here every rank
    gets the same count and the remainder is dropped;
  * communicator: one RCCL communicator per process, bootstrapped with a
    unique id that rank 0 creates and torch.distributed broadcasts (any
    backend: nccl on the GPU box, gloo in CPU tests);
  * host transport: the same Communicator with its two collectives carried
    by torch.distributed over gloo (host copies) — for ranks that share one
    GPU, where RCCL refuses two ranks on one device (tests, and the
    one-GPU rehearsal `NTS_BENCH_SHARE_GPU=1 bench.py --gpus N`).
"""
from __future__ import annotations

import numpy as np


def shard_nids(nids, world: int, rank: int):
    """Equal contiguous slice `rank` of `nids` (numpy array or torch tensor)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    per = len(nids) // world
    return nids[rank * per:(rank + 1) * per]


def steps_per_epoch(n_local: int, batch: int) -> int:
    return -(-n_local // batch)


def broadcast_unique_id(make_id, rank: int) -> bytes:
    """Rank 0 calls make_id() (128-byte RCCL id); every rank returns it."""
    import torch.distributed as dist
    obj = [make_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    uid = obj[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != 128:
        raise RuntimeError("RCCL unique id must be 128 bytes")
    return bytes(uid)


def make_communicator(ext, world: int, rank: int, local_rank: int):
    """nts_hip_comm (RCCL) for this process, or None for a single rank."""
    if world <= 1:
        return None
    uid = broadcast_unique_id(ext.Communicator.unique_id, rank)
    return ext.Communicator(world, rank, uid, local_rank)


def gloo_collective(tensor, op: int, root: int) -> None:
    """Communicator host transport over the default torch.distributed group:
    op 0 = SUM all-reduce in place, op 1 = broadcast from `root`."""
    import torch
    import torch.distributed as dist
    c = tensor.detach().cpu()
    if op == 0:
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    else:
        dist.broadcast(c, src=root)
    tensor.copy_(c)
    torch.cuda.synchronize()


def make_host_communicator(ext, world: int, rank: int, collective=gloo_collective):
    """The C++ driver's Communicator with a host transport (see module doc)."""
    return ext.Communicator.host(world, rank, collective)


def global_grad_sum(local_grads, all_reduce) -> list:
    """Reference Update() semantics: SUM (not mean) of every rank's W.grad
    (core/NtsScheduler.hpp:830-836).  `all_reduce` reduces one flat buffer in
    place — the fused single-collective form used by the C++ driver."""
    flat = np.concatenate([g.reshape(-1) for g in local_grads]).astype(np.float32)
    all_reduce(flat)
    out, off = [], 0
    for g in local_grads:
        out.append(flat[off:off + g.size].reshape(g.shape))
        off += g.size
    return out
