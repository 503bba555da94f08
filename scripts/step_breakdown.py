#!/usr/bin/env python3
"""Per-step kernel-time breakdown from a rocprofv3 kernel trace of bench.py.
usage: step_breakdown.py <run_kernel_trace.csv> [marker-substring] [nsteps]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mark = sys.argv[2] if len(sys.argv) > 2 else "k_spmm_gather<2, 64, 5, true>"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 5
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
a, b = idx[-n - 1], idx[-1]
wall = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3 / n
d = collections.defaultdict(lambda: [0, 0])
for r in rows[a:b]:
    k = r["Kernel_Name"].split("(")[0][:80]
    d[k][0] += 1
    d[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
tot = sum(v[1] for v in d.values()) / 1e3 / n
print(f"wall/step {wall:.1f} us, kernel-sum/step {tot:.1f} us")
for k, v in sorted(d.items(), key=lambda x: -x[1][1]):
    print(f"{v[0] / n:6.1f} x {v[1] / n / 1e3:8.1f} us  {k}")
