"""bench.py's reporting logic on CPU: the roofline picks the dominant kernel by
device time and divides its algorithmic units by the live average launch; a
committed PMC pass is attached only when it was taken on this very
libnts_hip.so build, kernel and workload (a stale pass is refused, with the
reason stated); the metric label follows the workload."""
import importlib.util
import json
import pathlib
import types

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _args(**kw):
    base = dict(shape="reddit", batch=10000, fanout="25-10", weight="sum", transform_first=-1,
                model="gcn", cache_rate=-1.0, gemm="split3", no_hip_gemm=False, no_pipeline=False,
                pd_cache=False, pd_rate=0.2, pd_super_batch=4, pair_table=0, rng="philox")
    base.update(kw)
    return types.SimpleNamespace(**base)


def test_roofline_dominant_kernel_and_units(bench, monkeypatch):
    monkeypatch.setattr(bench, "attach_pmc", lambda *a, **k: None)
    prof = {"bottom_aggregation": {"ms": 10.0, "calls": 20, "units": 20 * 0.87e9},
            "gat_forward": {"ms": 0.0, "calls": 0, "units": 0.0},
            "gather_gemm": {"ms": 2.0, "calls": 20, "units": 20 * 35e9}}
    rl = bench.roofline(prof, _args(), [602, 128, 41], 1)
    assert rl["kernel"] == "bottom_aggregation" and rl["bound"] == "hbm"
    assert rl["avg_launch_ms"] == pytest.approx(0.5)
    assert rl["achieved"] == pytest.approx(0.87e9 / 0.5e-3 / 1e9)
    assert rl["frac"] == pytest.approx(rl["achieved"] / bench.HBM_PEAK_GBS)
    assert rl["kernels"]["gather_gemm"]["bound"] == "mfma"
    assert "gat_forward" not in rl["kernels"]
    # f16 pair-table GEMM: three f16 MFMA products per fp32 product vs the f16
    # peak, its algorithmic bytes vs HBM; the larger fraction is the bound
    g = bench.roofline(prof, _args(pair_table=3), [602, 128, 41], 1)["kernels"]["gather_gemm"]
    rows = 35e9 / (2 * 602 * 128)
    assert g["f16_mfma_flops_per_launch"] == pytest.approx(3 * 35e9)
    assert g["algorithmic_bytes_per_launch"] == pytest.approx(rows * (4 * 608 + 4 * 128) + 4 * 608 * 128)
    assert g["mfma_frac"] == pytest.approx(3 * 35e9 / 0.1e-3 / 1e12 / bench.F16_MFMA_PEAK_TF)
    assert g["bound"] == "hbm" and g["frac"] == pytest.approx(max(g["mfma_frac"], g["hbm_frac"]))


def test_roofline_split3_gather_gemm_dual_roof(bench, monkeypatch):
    """fp32-exact gathered GEMM (csrc/gemmx3.hip): six bf16 MFMA products per
    fp32 product against the dense bf16 peak, its algorithmic bytes against
    HBM; the larger fraction is the reported bound; the dtype says fp32."""
    monkeypatch.setattr(bench, "attach_pmc", lambda *a, **k: None)
    prof = {"gather_gemm_tn": {"ms": 4.0, "calls": 20, "units": 20 * 35e9}}
    rl = bench.roofline(prof, _args(), [602, 128, 41], 1)
    g = rl["kernels"]["gather_gemm_tn"]
    rows = 35e9 / (2 * 602 * 128)
    assert g["bf16_mfma_flops_per_launch"] == pytest.approx(6 * 35e9)
    assert g["algorithmic_bytes_per_launch"] == pytest.approx(rows * (4 * 608 + 4 * 128) + 4 * 608 * 128)
    assert g["mfma_frac"] == pytest.approx(6 * 35e9 / 0.2e-3 / 1e12 / bench.F16_MFMA_PEAK_TF)
    assert g["frac"] == pytest.approx(max(g["mfma_frac"], g["hbm_frac"]))
    assert rl["kernel"] == "gather_gemm_tn"
    assert bench.dtype_name(_args(), True).startswith("fp32 ")
    assert "narrower than fp32" in bench.dtype_name(_args(pair_table=3), True)


def test_pmc_attached_only_for_the_same_build_and_workload(bench, monkeypatch, tmp_path):
    (tmp_path / "profiles").mkdir()
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    monkeypatch.setattr(bench, "lib_sha256", lambda: "abc")
    args, layers = _args(), [602, 128, 41]
    wl = bench.pmc_workload(args, layers, 1)
    info = {"workload": wl, "lib_sha256": "abc", "profiler_kernel": "bottom_aggregation",
            "kernels": {"k": {"profiler_kernel": "bottom_aggregation",
                              "hbm_bytes_per_launch": 3.75e9}}}
    (tmp_path / "profiles" / "pmc_x.json").write_text(json.dumps(info))
    rl = {"avg_launch_ms": 0.5}
    bench.attach_pmc(rl, "bottom_aggregation", args, layers, 1)
    assert rl["traffic"] == pytest.approx(3.75e9)
    assert rl["traffic_GBs"] == pytest.approx(3.75e9 / 0.5e-3 / 1e9)
    # another build: refused, reason stated
    info["lib_sha256"] = "old"
    (tmp_path / "profiles" / "pmc_x.json").write_text(json.dumps(info))
    rl = {"avg_launch_ms": 0.5}
    bench.attach_pmc(rl, "bottom_aggregation", args, layers, 1)
    assert "traffic" not in rl and "another libnts_hip.so build" in rl["traffic_note"]
    # another workload: not attached
    info["lib_sha256"] = "abc"
    (tmp_path / "profiles" / "pmc_x.json").write_text(json.dumps(info))
    rl = {"avg_launch_ms": 0.5}
    bench.attach_pmc(rl, "bottom_aggregation", _args(batch=1024), layers, 1)
    assert "traffic" not in rl


def test_metric_and_workload_labels(bench):
    assert "2-hop GCN on Reddit-shaped" in bench.metric_name(_args(), [602, 128, 41])
    assert "3-hop GraphSAGE on ogbn-products-shaped" in bench.metric_name(
        _args(shape="products", weight="mean"), [100, 256, 256, 47])
    w = bench.workload_name(_args(), [602, 128, 41], 232965, 114848857, False)
    assert "split-bf16" in w and "fused gather/aggregation" in w


def _run_bench(args, **env_extra):
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")
           and not k.startswith("NTS_")}
    env.update(env_extra)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True,
                          text=True, env=env, timeout=300)


def test_gpus_n_launches_n_ranks_itself():
    """bench.py --gpus 2 with no launcher starts torch.distributed.run as a
    child, every rank joins, and the parent relays rank 0's line."""
    r = _run_bench(["--gpus", "2", "--launch-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    obj = json.loads(lines[0])
    assert obj["n_gpus"] == 2 and sorted(obj["ranks"]) == [0, 1]
    assert "torch.distributed.run" in obj["config"]["launcher"]
    # an N-rank line carries the communicator's rank count and the
    # gradient exchange's own time per step
    assert "rccl_ranks" in obj and obj["config"]["allreduce_us_per_step"] > 0


def test_world_size_must_match_gpus():
    r = _run_bench(["--gpus", "1", "--launch-selftest"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in r.stderr


def test_diagnostic_knobs_are_refused():
    r = _run_bench(["--launch-selftest"], NTS_NN3_DIAG="1")
    assert r.returncode != 0 and "NTS_NN3_DIAG" in r.stderr
    r = _run_bench(["--launch-selftest"], NTS_DIAG_REUSE_SAMPLE="1")
    assert r.returncode != 0 and "NTS_DIAG_REUSE_SAMPLE" in r.stderr


def test_nts_env_is_recorded(bench, monkeypatch):
    monkeypatch.setenv("NTS_MT_SERIAL", "1")
    monkeypatch.setenv("NTS_SCAN1", "0")  # a former knob, now a compile-time flag
    env = bench.nts_env()
    assert env["NTS_MT_SERIAL"] == "1" and "NTS_SCAN1" not in env
    assert env["ignored"] == ["NTS_SCAN1"]
    assert bench.diag_env() == []


def test_child_argv_keeps_the_workload(bench):
    """A secondary child runs the parent's own workload: every
    workload flag given to the parent (--rng, --no-pad-features, --cache-rate
    ...) reaches the child, the secondary controls do not, and the overrides
    replace the parent's value of the same flag."""
    argv = ["--rng", "mt", "--no-pad-features", "--cache-rate", "0.3", "--steps", "7",
            "--transform-first=1", "--no-secondary-mt", "--gpus", "1", "--cpu-threads", "4",
            "--epochs", "2", "--sampler-gate", "1"]
    out = bench.child_argv(argv, {"--transform-first": 0, "--pair-table": 0})
    assert out[:7] == ["--rng", "mt", "--no-pad-features", "--cache-rate", "0.3", "--steps", "7"]
    assert "--transform-first=1" not in out and out.count("--transform-first") == 1
    assert out[out.index("--transform-first") + 1] == "0" and out[out.index("--pair-table") + 1] == "0"
    for gone in ("--no-secondary-mt", "--gpus", "--cpu-threads", "--epochs"):
        assert gone not in out
    assert out[-1] == "--secondary" and out[out.index("--sampler-gate") + 1] == "1"
    mt = bench.child_argv(["--rng", "philox", "--no-pad-features"], {"--rng": "mt"})
    assert mt == ["--no-pad-features", "--rng", "mt", "--secondary"]


def test_product_library_env_knobs():
    """The product library reads at most these environment variables (the
    A/B variants are compile-time flags of `make variant`, the timing probes
    exist only in `make probe`): a debugging aid for hangs and the two
    MT19937 walker selections the kernel tests A/B."""
    import re
    lib = ROOT / "sample-based-gnn_amd" / "nts" / "lib" / "libnts_hip.so"
    if not lib.exists():
        pytest.skip("libnts_hip.so not built")
    names = set(m.group(1).decode() for m in re.finditer(rb"\x00(NTS_[A-Z0-9_]+)\x00", lib.read_bytes()))
    assert names <= {"NTS_LAUNCH_TRACE", "NTS_MT_SERIAL", "NTS_MT_CHUNKED"}, names
    assert len(names) <= 10


def test_host_extension_env_knobs():
    """The C++ host layer reads only two timing aids (NTS_TF_* /
    NTS_TN_CHUNK_SCALES are compile-time A/B flags since round 6)."""
    import re
    ext = ROOT / "sample-based-gnn_amd" / "nts" / "lib" / "host_build" / "nts_host_ext.so"
    if not ext.exists():
        pytest.skip("nts_host_ext.so not built")
    names = set(m.group(1).decode() for m in re.finditer(rb"\x00(NTS_[A-Z0-9_]+)\x00", ext.read_bytes()))
    assert names <= {"NTS_HOST_PROFILE", "NTS_TIMELINE"}, names
