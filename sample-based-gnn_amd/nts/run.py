"""`nts <cfg>`: run a training job from a reference configuration file.

Mirrors the reference's entry point (toolkits/main.cpp:59-186): read the cfg
(InputInfo::readFromCfgFile, core/GraphSegment.cpp:222-347), load the graph
and the vertex data, pick the driver by ALGORITHM, and run EPOCHS epochs of
train + eval + test with the reference's per-epoch report
(toolkits/GCN_SAMPLE_ALLGPU.hpp:361-383, 467-482).  Every ALGORITHM runs on
the MI355X path of this build; the mapping is:

  GCNSAMPLESINGLE  (GCN_CPU_SAMPLE)   GCN, the reference's mt19937 neighbour
                                      stream and bias-corrected Adam
                                      (learnC2C_with_decay_Adam), on the GPU
  GCNSAMPLEGPU / GCNSAMPLEALLGPU      GCN, Philox sampler, GPU Adam
  GSSAMPLEALLGPU                      the same pipeline with Mean weights
                                      (SURVEY B-5: the reference GPU toolkit
                                      actually runs Sum; MEAN_WEIGHT:gpu selects
                                      its get_mean_weight formula)
  GCNSAMPLEALLMULTI                   data parallel: launch one process per GPU
                                      with torch.distributed.run
  GCNSAMPLEPDCACHE / GSSAMPLEPDCACHE  GCN / GraphSAGE with the NeutronOrch PD
                                      cache: super-batches of PIPELINE_NUM
                                      batches, CACHE_RATE hot vertices each
                                      (preSample; PRE_SAMPLE_FILE read, or
                                      written when missing); with
                                      FEATURE_CACHE_RATE the feature table
                                      moves to pinned host memory with that
                                      fraction cached in HBM
  GATSAMPLEALLGPU                     GAT

Usage:  python -m nts.run path/to/job.cfg [--epochs N] [--device D] [--json out.json]
File paths inside the cfg are resolved relative to the cfg's directory.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

import numpy as np
import torch

from . import dataloader

ALGORITHMS = {
    # name: (model, weight, rng, bias_correction, feature placement)
    "GCNSAMPLESINGLE": ("gcn", "sum", "mt", True, None),
    # GCN_SAMPLE_GPU: sample_fast's mt19937 stream (replayed on the device) ->
    # SingleGPUSampleGraphOp (CSR backward), GPU Adam (toolkits/GCN_SAMPLE_GPU.hpp:289-394)
    "GCNSAMPLEGPU": ("gcn", "sum", "mt", False, "sample_gpu"),
    "GCNSAMPLEALLGPU": ("gcn", "sum", "philox", False, None),
    "GSSAMPLEALLGPU": ("gcn", "mean", "philox", False, None),
    "GCNSAMPLEALLMULTI": ("gcn", "sum", "philox", False, None),
    "GCNSAMPLEPDCACHE": ("gcn", "sum", "philox", False, "pd"),
    "GSSAMPLEPDCACHE": ("gcn", "mean", "philox", False, "pd"),
    "GATSAMPLEALLGPU": ("gat", "none", "philox", False, None),
}


def _path(base: pathlib.Path, p: str) -> pathlib.Path:
    q = pathlib.Path(p)
    return q if q.is_absolute() else (base / q)


def load_inputs(info: dataloader.InputInfo, base: pathlib.Path, n_classes: int, device=None):
    """Edge list (binary u32 pairs; with `device`, streamed in chunks straight
    into int32 device tensors), features/labels/masks (text or
    FEATURE_FILE:random)."""
    if device is None:
        src, dst = dataloader.read_edge_file(_path(base, info.edge_file))
    else:
        src, dst = dataloader.load_edges_to_device(_path(base, info.edge_file), device)
    V = info.vertices
    F = info.layers[0]
    if info.feature_file in ("", "random"):
        feats, labels, masks = dataloader.random_generate(V, F, n_classes)
    else:
        fpath = _path(base, info.feature_file)
        if not fpath.exists() and pathlib.Path(str(fpath) + ".zip").exists():
            fpath = pathlib.Path(str(fpath) + ".zip")
        feats, labels, masks = dataloader.read_feature_label_mask(
            fpath, _path(base, info.label_file), _path(base, info.mask_file), V, F)
    return src, dst, feats, labels, masks


def build_driver(E, info: dataloader.InputInfo, G, feat, labels, train_ids, device, comm=None):
    from . import host, _abi
    algo = info.algorithm.upper()
    if algo not in ALGORITHMS:
        raise SystemExit(f"ALGORITHM {info.algorithm}: not supported by this build "
                         f"(supported: {', '.join(sorted(ALGORITHMS))})")
    model, weight, rng, bias, place = ALGORITHMS[algo]
    if weight == "mean" and info.extra.get("MEAN_WEIGHT", "").lower() == "gpu":
        weight = "mean-sampled"
    cache_rate = -1.0
    pd = place == "pd"
    if pd and "FEATURE_CACHE_RATE" in info.extra:
        cache_rate = float(info.extra["FEATURE_CACHE_RATE"])
    cfg = host.gcn_config(
        info.layers, info.fanout, info.batch_size, learn_rate=info.learn_rate,
        weight_decay=info.weight_decay, drop_rate=info.drop_rate,
        rng_mode=_abi.NTS_RNG_MT19937_LEMIRE if rng == "mt" else _abi.NTS_RNG_PHILOX,
        weight="none" if model == "gat" else weight, bias_correction=bias,
        pipeline=info.pipeline_num > 1, up_degree=info.up_degree, gat=model == "gat",
        cache_rate=cache_rate, shuffle=True, pd_cache=pd, pd_rate=info.cache_rate,
        pd_super_batch=max(info.pipeline_num, 1), sample_gpu=place == "sample_gpu")
    return E.GCN_SAMPLE_ALLGPU_impl(G, feat, labels, train_ids, cfg, comm)


def pd_presample_file(drv, info, base, out=print, rank=0, world=1):
    """PRE_SAMPLE_FILE (core/ntsBaseOp.hpp:427-497): read the hot vertices of
    every super-batch if the file exists, else keep the device preSample the
    driver ran and write it (default name when the key is unset).  Under
    WORLD_SIZE > 1 each rank has its own train shard and so its own file
    (`.rank<r>` appended): no two ranks write one path."""
    name = info.pre_sample_file or dataloader.presample_file_name(
        _path(base, info.edge_file), info.batch_size, info.fanout_string, info.pipeline_num)
    path = _path(base, name)
    if world > 1:
        path = path.with_name(path.name + f".rank{rank}")
    counts, ids = drv.presample()
    if path.exists():
        kc, kids = dataloader.read_presample_file(path, len(counts))
        drv.set_presample(kc.tolist(), kids.tolist())
        out(f"pre sample file: {path} (read, {len(kc)} super-batches, {kids.size} hot vertices)")
    else:
        try:
            dataloader.write_presample_file(path, counts, ids)
            out(f"pre sample file: {path} (written, {len(counts)} super-batches, {len(ids)} hot vertices)")
        except OSError:
            out(f"pre sample file: {path} not writable; using the device preSample")


def run(cfg_path, epochs=None, device=0, out=print) -> dict:
    from . import host
    from . import dist as ndist
    cfg_path = pathlib.Path(cfg_path)
    info = dataloader.InputInfo.from_cfg(cfg_path)
    base = cfg_path.parent
    n_classes = info.layers[-1]
    epochs = info.epochs if epochs is None else epochs
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", device))
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    E = host.ext()
    t0 = time.time()
    src, dst, feats, labels, masks = load_inputs(info, base, n_classes, device=dev)
    G = E.FullyRepGraph.from_edges(src, dst, info.vertices)
    n_edges = src.numel()
    del src, dst
    feat = torch.from_numpy(feats).to(dev)
    lab = torch.from_numpy(labels).to(dev)
    ids = {k: np.nonzero(masks == v)[0].astype(np.int32) for k, v in
           (("train", dataloader.MASK_TRAIN), ("val", dataloader.MASK_VAL),
            ("test", dataloader.MASK_TEST))}
    train = torch.from_numpy(ndist.shard_nids(ids["train"], world, rank))
    comm = ndist.make_communicator(E, world, rank, device)
    drv = build_driver(E, info, G, feat, lab, train, dev, comm)
    if ALGORITHMS.get(info.algorithm.upper(), ("",) * 5)[4] == "pd":
        pd_presample_file(drv, info, base, out if rank == 0 else (lambda s: None), rank, world)
    if rank == 0:
        out(f"GNNmini::Engine[MI355X.GPU.{info.algorithm}] running [{epochs}] Epochs "
            f"(V={info.vertices}, E={n_edges}, layers {info.layer_string}, fanout "
            f"{info.fanout_string}, batch {info.batch_size}; loaded in {time.time() - t0:.1f}s)")
    hist = []
    for ep in range(epochs):
        te = time.perf_counter()
        drv.reset_correct()
        drv.run_epoch()
        correct = drv.train_correct()  # synchronises
        loss = float(drv.loss.detach().cpu())
        t_train = time.perf_counter() - te
        acc_val = drv.evaluate(torch.from_numpy(ids["val"])) if ids["val"].size else 0.0
        acc_test = drv.evaluate(torch.from_numpy(ids["test"])) if ids["test"].size else 0.0
        n_train = int(train.numel())
        rec = {"epoch": ep, "train_acc": correct / max(n_train, 1), "train_correct": int(correct),
               "n_train": n_train, "eval_acc": acc_val, "test_acc": acc_test, "loss": loss,
               "epoch_time_s": time.perf_counter() - te, "train_time_s": t_train}
        hist.append(rec)
        if rank == 0:
            out(f"Train Acc: {rec['train_acc']:f} {correct} {n_train}")
            out(f"Eval Acc: {acc_val:f} {int(round(acc_val * ids['val'].size))} {ids['val'].size}")
            out(f"Test Acc: {acc_test:f} {int(round(acc_test * ids['test'].size))} {ids['test'].size}")
            out(f"GNNmini::Running.Epoch[{ep}]:Times[{rec['epoch_time_s']:f}(s)]:loss\t{loss:f}")
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return {"cfg": str(cfg_path), "algorithm": info.algorithm, "epochs": hist}


def main(argv=None):
    p = argparse.ArgumentParser(prog="nts", description=__doc__.split("\n")[0])
    p.add_argument("cfg")
    p.add_argument("--epochs", type=int, default=None)
    p.add_argument("--device", type=int, default=int(os.environ.get("LOCAL_RANK", "0")))
    p.add_argument("--json", default=None)
    a = p.parse_args(argv)
    res = run(a.cfg, a.epochs, a.device)
    if a.json:
        pathlib.Path(a.json).write_text(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
