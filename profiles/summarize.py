#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run into committed artefacts.

  python profiles/summarize.py <gpurun_out/prof_TAG> <TAG>

Writes profiles/<TAG>_kernel_stats.csv (rocprofv3 --stats, as produced),
profiles/<TAG>_summary.md (top kernels, the bench line's live HIP-event
averages next to the trace's, PMC traffic) and profiles/pmc_<TAG>.json: per
profiled kernel the HBM bytes per launch = FETCH_SIZE x 2 (gfx950 tallies
128-B requests at 64 B, MI355X_MICROARCH.md §HBM) + WRITE_SIZE (both KiB per
dispatch), tagged with the libnts_hip.so sha256 and the workload the bench
line reports, so bench.py attaches it only to the same build and workload.
"""
import csv
import json
import pathlib
import re
import shutil
import statistics
import sys

# bench profiler kernel -> how its HIP kernel reads in a rocprofv3 trace
def profiler_kernel(name: str):
    if "nts_hip::k_gat_fwd" in name:
        return "gat_forward"
    m = re.search(r"nts_hip::(\w+)<([^>]*)>", name)
    if not m:
        return None
    k, targs = m.group(1), [a.strip() for a in m.group(2).split(",")]
    if k == "k_spmm_gather":
        mode = targs[6] if len(targs) > 6 else "0"
        if mode == "1":
            return "bottom_aggregation"          # transform-first: A H + relu/dropout
        if mode in ("2", "4"):
            return "bottom_backward"             # A^T (dX ⊙ mask) / A^T dZ + column maxima
        if targs[3] == "true" and targs[5] == "false":
            return "bottom_aggregation"          # aggregate-first: fused gather A X
        return None
    if k == "k_gemm_wres" and targs[2] == "false":
        return "gather_gemm"                     # X[src] W0 (no epilogue)
    if k == "k_gemm3_nn" and targs == ["false", "true"]:
        return "gather_gemm"                     # split-bf16 X[src] W0
    if k == "k_x3_nn" and targs[0] == "false":
        return "gather_gemm"                     # split-bf16 X[src] W0, whole rows (gemmx3.hip)
    if k == "k_x3_nn7" and len(targs) > 2 and targs[2] == "false":
        return "gather_gemm"                     # round 6: 4-wave blocks, 7 row tiles a wave
    if k == "k_x3_tn":
        return "gather_gemm_tn"                  # split-bf16 X[src]^T dH, whole rows (gemmx3.hip)
    if k == "k_gemm_tn_big" and targs[0] == "false":
        return "gather_gemm_tn"                  # X[src]^T dH (no mask)
    if k == "k_s3_tn" and targs[1:] == ["false", "true"]:
        return "gather_gemm_tn"                  # split-bf16 X[src]^T dH
    if k in ("k_h2_nn", "k_h2_nn2", "k_h2_nn3") and targs[:2] == ["false", "true"]:
        return "gather_gemm"                     # f16 pair table X[src] W0
    if k in ("k_h2_tn2", "k_h2_tn3", "k_h2_tn4"):
        return "gather_gemm_tn"                  # f16 pair table X[src]^T dH
    return None


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def bench_line(log):
    for line in reversed(pathlib.Path(log).read_text().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def main():
    src = pathlib.Path(sys.argv[1])
    tag = sys.argv[2]
    dst = pathlib.Path(__file__).resolve().parent
    stats = next(src.glob("trace/**/run_kernel_stats.csv"))
    shutil.copy(stats, dst / f"{tag}_kernel_stats.csv")
    rows = load(stats)
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    bl = bench_line(src / "trace.log")
    meta = (bl or {}).get("config", {}).get("profile_meta", {})
    lines = [f"# rocprofv3 summary — {tag}", "",
             f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py {meta.get('argv', '')}` "
             f"(the trace includes graph generation / CSC build before the timed steps).", "",
             "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.3f} | "
                     f"{float(r['AverageNs'])/1e3:.1f} | {100*float(r['TotalDurationNs'])/tot:.1f} |")
    info = {"workload": meta.get("workload"), "lib_sha256": meta.get("lib_sha256"),
            "profiler_kernel": (bl or {}).get("roofline", {}).get("kernel"), "kernels": {}}
    live = (bl or {}).get("roofline", {}).get("kernels", {})
    for r in rows:
        pk = profiler_kernel(r["Name"])
        if pk is None:
            continue
        cur = info["kernels"].get(r["Name"])
        info["kernels"][r["Name"]] = {"profiler_kernel": pk, "avg_ns": float(r["AverageNs"]),
                                      "calls": int(r["Calls"])}
    counters = (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE"), ("hit", "TCC_HIT_sum"),
                ("hit", "TCC_MISS_sum"))
    for kind, counter in counters:
        p = list(src.glob(f"{kind}/**/run_counter_collection.csv"))
        if not p:
            continue
        per = {}
        for r in load(p[0]):
            if r.get("Counter_Name") == counter:
                per.setdefault(r["Kernel_Name"].split("(")[0].strip(), []).append(float(r["Counter_Value"]))
        for name, kv in info["kernels"].items():
            vals = per.get(name.split("(")[0].strip())
            if vals:
                kv[counter] = statistics.median(vals)  # KiB per dispatch (median over launches)
    lines += ["", "## Profiled kernels (bench `roofline.kernels`, live HIP events) vs the trace", "",
              "| bench kernel | HIP kernel | live avg us | trace avg us | HBM GB/launch (PMC) | L2 hit |",
              "|---|---|---|---|---|---|"]
    for name, kv in info["kernels"].items():
        if "FETCH_SIZE" in kv and "WRITE_SIZE" in kv:
            kv["hbm_bytes_per_launch"] = (2 * kv["FETCH_SIZE"] + kv["WRITE_SIZE"]) * 1024.0
        if "TCC_HIT_sum" in kv and "TCC_MISS_sum" in kv:
            kv["l2_hit_rate"] = kv["TCC_HIT_sum"] / max(kv["TCC_HIT_sum"] + kv["TCC_MISS_sum"], 1.0)
        lk = live.get(kv["profiler_kernel"], {})
        alg = lk.get("algorithmic_bytes_per_launch")
        if alg and "hbm_bytes_per_launch" in kv:
            kv["traffic_over_algorithmic"] = kv["hbm_bytes_per_launch"] / alg
        lines.append(
            f"| {kv['profiler_kernel']} | `{name.split('(')[0][:70]}` | "
            f"{lk.get('avg_launch_ms', float('nan')) * 1e3:.1f} | {kv['avg_ns'] / 1e3:.1f} | "
            f"{kv.get('hbm_bytes_per_launch', float('nan')) / 1e9:.3f} | "
            f"{kv.get('l2_hit_rate', float('nan')):.3f} |")
        if "traffic_over_algorithmic" in kv:
            lines.append(f"|  | counter / algorithmic bytes: {kv['traffic_over_algorithmic']:.2f} | | | | |")
    # engine counters of the heaviest kernels (own pass: SQ / GRBM)
    sqp = list(src.glob("sq/**/run_counter_collection.csv"))
    if sqp:
        per = {}
        for r in load(sqp[0]):
            per.setdefault(r["Kernel_Name"].split("(")[0].strip(), {}).setdefault(
                r["Counter_Name"], []).append(float(r["Counter_Value"]))
        lines += ["", "## Engine counters (own rocprofv3 --pmc pass; medians per dispatch)", "",
                  "MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); "
                  "clock = GRBM_GUI_ACTIVE / 8 / trace duration (MI355X_MICROARCH.md: DVFS); "
                  "wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES.", "",
                  "| kernel | trace avg us | MFMA busy | clock GHz | wave wait | LDS bank-conflict cycles |",
                  "|---|---|---|---|---|---|"]
        engine = {}
        for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
            c = per.get(r["Name"].split("(")[0].strip())
            if not c:
                continue
            med = {k: statistics.median(v) for k, v in c.items()}
            gui = med.get("GRBM_GUI_ACTIVE", 0.0)
            avg_us = float(r["AverageNs"]) / 1e3
            busy = med.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (128.0 * gui) if gui else float("nan")
            clk = gui / 8.0 / (avg_us * 1e3) if avg_us else float("nan")
            wait = med.get("SQ_WAIT_ANY", 0.0) / med["SQ_WAVE_CYCLES"] if med.get("SQ_WAVE_CYCLES") else float("nan")
            engine[r["Name"]] = {"mfma_busy": busy, "clock_ghz": clk, "wave_wait": wait,
                                 "lds_bank_conflict_cycles": med.get("SQ_LDS_BANK_CONFLICT")}
            lines.append(f"| `{r['Name'].split('(')[0][:70]}` | {avg_us:.1f} | {busy:.2f} | {clk:.2f} | "
                         f"{wait:.2f} | {med.get('SQ_LDS_BANK_CONFLICT', float('nan')):.3g} |")
        info["engine"] = engine
    if bl:
        lines += ["", f"Bench line of the traced run: value {bl['value']:.4g} {bl['unit']}, "
                      f"{bl['ms_per_step']:.3f} ms/step (profiled: slower than un-profiled)."]
    (dst / f"{tag}_summary.md").write_text("\n".join(lines) + "\n")
    (dst / f"pmc_{tag}.json").write_text(json.dumps(info, indent=1) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
