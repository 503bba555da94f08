#!/usr/bin/env python3
"""Average duration per kernel over the last N steps of a rocprofv3 trace.
usage: kernel_avg.py <run_kernel_trace.csv> [nsteps] [filter-substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
flt = sys.argv[3] if len(sys.argv) > 3 else ""
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_spmm_gather<2, 64, 5, true" in r["Kernel_Name"]]
a, b = idx[-n - 1], idx[-1]
d = collections.defaultdict(list)
for r in rows[a:b]:
    d[r["Kernel_Name"].split("(")[0][:70]].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if flt in k:
        v.sort()
        print(f"{len(v)/n:4.1f}x  mean {sum(v)/len(v):7.1f}  min {v[0]:7.1f}  med {v[len(v)//2]:7.1f}  {k}")
