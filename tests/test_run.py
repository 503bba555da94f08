"""The cfg-driven entry point (`nts <cfg>`, toolkits/main.cpp:59-186) on the
reference's own Cora job (gcn_cora_sample.cfg: 1433-256-7, fanout 25-10,
batch 64, lr 0.01, dropout 0.5, 10 epochs) and data files.

The only reference-produced output on this path is the Cora training log
(log/cora_gcn/output.log:67-158): train accuracy 0.765 at epoch 0 rising to
0.929 at epoch 9.  It comes from the GCN_SAMPLE_PD_CACHE toolkit with its own
random streams, so it is a loose sanity bound on the learning behaviour, not
parity: the test asks for the same regime (>= 0.88 train accuracy by the last
epoch, rising from the first epoch).
"""
import numpy as np
import pytest

from conftest import GOLDEN
from nts import dataloader

CFG = GOLDEN / "cora" / "gcn_cora_sample.cfg"


def test_cfg_parses_reference_job():
    info = dataloader.InputInfo.from_cfg(CFG)
    assert info.algorithm == "GCNSAMPLEALLGPU"
    assert (info.vertices, info.layers, info.fanout, info.batch_size, info.epochs) == (
        2708, [1433, 256, 7], [25, 10], 64, 10)
    assert (info.learn_rate, info.weight_decay, info.drop_rate, info.pipeline_num) == (
        0.01, 0.0001, 0.5, 4)


def test_runner_loads_cora_inputs():
    from nts import run
    info = dataloader.InputInfo.from_cfg(CFG)
    src, dst, feats, labels, masks = run.load_inputs(info, CFG.parent, 7)
    assert src.size == 13566 and feats.shape == (2708, 1433)
    assert set(np.unique(labels)) <= set(range(7))
    assert (masks == dataloader.MASK_TRAIN).sum() == 1605  # the log's "... 1605"
    assert feats.sum() > 0


@pytest.mark.gpu
def test_cora_job_trains_like_the_reference_log():
    from nts import run
    lines = []
    res = run.run(CFG, out=lines.append)
    acc = [e["train_acc"] for e in res["epochs"]]
    assert len(acc) == 10
    assert acc[-1] >= 0.88, acc
    assert acc[-1] > acc[0], acc
    assert 0.5 <= res["epochs"][-1]["test_acc"] <= 1.0
    assert any(l.startswith("Train Acc:") for l in lines)
    assert res["epochs"][-1]["n_train"] == 1605


@pytest.mark.gpu
def test_gcn_cpu_sample_algorithm_runs_mt19937_and_bias_corrected_adam():
    """ALGORITHM:GCNSAMPLESINGLE maps to GCN_CPU_SAMPLE's semantics on the GPU:
    the reference's mt19937 neighbour stream and learnC2C_with_decay_Adam."""
    import shutil
    import tempfile
    import pathlib
    from nts import run
    d = pathlib.Path(tempfile.mkdtemp())
    for f in ("cora.2708.edge.self", "cora.featuretable.zip", "cora.labeltable", "cora.mask"):
        shutil.copy(GOLDEN / "cora" / f, d / f)
    text = CFG.read_text().replace("ALGORITHM:GCNSAMPLEALLGPU", "ALGORITHM:GCNSAMPLESINGLE")
    (d / "job.cfg").write_text(text)
    res = run.run(d / "job.cfg", epochs=3, out=lambda s: None)
    assert res["epochs"][-1]["train_acc"] > 0.5


@pytest.mark.gpu
def test_pd_cache_cora_job_and_presample_file(tmp_path):
    """The reference's own job (ALGORITHM:GCNSAMPLEPDCACHE, CACHE_RATE 0.2,
    PIPELINE_NUM 4): trains with the PD cache, writes the PRE_SAMPLE_FILE on
    the first run and reads it back on the second with the same result."""
    import shutil
    from nts import run
    for f in ("cora.2708.edge.self", "cora.featuretable.zip", "cora.labeltable", "cora.mask"):
        shutil.copy(GOLDEN / "cora" / f, tmp_path / f)
    text = CFG.read_text().replace("ALGORITHM:GCNSAMPLEALLGPU", "ALGORITHM:GCNSAMPLEPDCACHE")
    (tmp_path / "job.cfg").write_text(text + "PRE_SAMPLE_FILE:hot.bin\n")
    lines = []
    r1 = run.run(tmp_path / "job.cfg", epochs=4, out=lines.append)
    assert (tmp_path / "hot.bin").exists() and any("written" in l for l in lines)
    lines2 = []
    r2 = run.run(tmp_path / "job.cfg", epochs=4, out=lines2.append)
    assert any("(read" in l for l in lines2)
    assert [e["train_correct"] for e in r1["epochs"]] == [e["train_correct"] for e in r2["epochs"]]
    assert r1["epochs"][-1]["train_acc"] > 0.7
