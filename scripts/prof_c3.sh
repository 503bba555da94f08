#!/bin/bash
# rocprofv3 kernel trace + stats of a short C3 (products-shaped GraphSAGE,
# 100-256-256-47, 15-10-5, B=1024) bench run; per-kernel time per step.
export TMPDIR=/tmp
O=gpurun_out/${1:-c3p}
mkdir -p $O
shift || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 bench.py --shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean --steps 40 --warmup 5 --no-cpu-baseline --epochs 0 --sampler-batches 0 --no-secondary-af "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 - "$O" 40 <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
steps = int(sys.argv[2])
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
L = 3
a, b = adam[-(steps * L) - 1], adam[-1]
win = rows[a + 1:b + 1]
t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
for r in win:
    n = r["Kernel_Name"].split("(")[0][:90]
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("window %.1f us over %d steps = %.1f us/step, %d kernels" % ((t1 - t0) / 1e3, steps, (t1 - t0) / 1e3 / steps, len(win)))
tot = sum(d for c, d in agg.values())
print("sum of kernel time per step %.1f us" % (tot / steps))
for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
    print("%8.1f us/step  x%-5.1f %s" % (d / steps, c / steps, n))
PY
