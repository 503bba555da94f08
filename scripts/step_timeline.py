#!/usr/bin/env python3
"""Kernel-by-kernel timeline of one training step on the training queue.
usage: step_timeline.py <run_kernel_trace.csv> [marker]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mark = sys.argv[2] if len(sys.argv) > 2 else "k_spmm_gather<2, 64, 5, true>"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b + 1]:
    if r["Queue_Id"] != rows[a]["Queue_Id"]:
        continue
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{s:8.1f} {d:7.1f}  grid {r['Grid_Size_X']:>8} x {r['Workgroup_Size_X']:>4}  "
          f"{r['Kernel_Name'][:64]}")
