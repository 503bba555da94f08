#!/bin/bash
# rocprofv3 kernel trace of the GPU sampler running alone (bench.py's
# sampler-only phase: 32 batches after one training step)
export TMPDIR=/tmp
O=gpurun_out/${1:-samp1}
mkdir -p $O
shift || true
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --epochs 0 --sampler-batches 32 --no-secondary-af --no-secondary-exact --no-interference-probe "$@" > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the sampler-only phase: after the last training-step kernel (k_adam)
last = max(i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"])
win = rows[last + 1:]
t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
for r in win:
    n = r["Kernel_Name"].split("(")[0][:80]
    agg[n][0] += 1
    agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("sampler-only window %.1f us, %d kernels" % ((t1 - t0) / 1e3, len(win)))
for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:20]:
    print("%9.1f us  x%-4d %s" % (d, c, n))
PY
