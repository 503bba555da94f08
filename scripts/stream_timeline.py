#!/usr/bin/env python3
"""Per-queue busy time per step from a rocprofv3 kernel trace of bench.py
(which kernels ran on which queue, and how much of the step each queue was busy).
usage: stream_timeline.py <run_kernel_trace.csv> [marker] [nsteps]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mark = sys.argv[2] if len(sys.argv) > 2 else "k_spmm_gather<2, 64, 5, true>"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 5
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
a, b = idx[-n - 1], idx[-1]
t0, t1 = int(rows[a]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
print(f"wall/step {(t1 - t0) / 1e3 / n:.1f} us")
q = collections.defaultdict(list)
for r in rows[a:b]:
    q[r["Queue_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
for qid, ks in q.items():
    # union of busy intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in sorted(ks):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = collections.Counter()
    for s, e, k in ks:
        tot[k.split("(")[0][-60:]] += e - s
    print(f"queue {qid}: {len(ks) / n:.0f} kernels/step, busy {busy / 1e3 / n:.1f} us/step")
    for k, v in tot.most_common(8):
        print(f"    {v / 1e3 / n:8.1f} us  {k}")
