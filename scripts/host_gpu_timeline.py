#!/usr/bin/env python3
"""Host API calls next to GPU kernel times for one bench step (rocprofv3
--kernel-trace --hip-runtime-trace output).  Shows where the host blocks.
usage: host_gpu_timeline.py <dir> [min_us]"""
import csv
import sys

d = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
ks = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
api = list(csv.DictReader(open(f"{d}/run_hip_api_trace.csv")))
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(ks) if "k_spmm_gather<2, 64, 5, true>" in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
t0, t1 = int(ks[a]["Start_Timestamp"]), int(ks[b]["Start_Timestamp"])
print(f"step {(t1 - t0) / 1e3:.1f} us (GPU time 0 = bottom gather of step k)")
corr = {r["Correlation_Id"]: r for r in ks}
rows = []
for r in api:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 - 1500000 < s < t1 + 100000:
        rows.append((s, e, r["Function"], r["Correlation_Id"]))
for s, e, f, c in sorted(rows):
    k = corr.get(c)
    if (e - s) / 1e3 >= min_us or (k and int(k["End_Timestamp"]) - int(k["Start_Timestamp"]) > 100000):
        kn = ""
        if k:
            kn = f"{k['Kernel_Name'].split('(')[0][-34:]} @gpu {(int(k['Start_Timestamp']) - t0) / 1e3:.0f}"
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {f:24s} {kn}")
