#!/bin/bash
# Kernel trace of the C2 bench with the reference's MT19937 stream (--rng mt).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04mtp}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 --rng mt --steps 10 --warmup 2 --no-interference-probe > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/tr <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print("%10.1f us  x%-5s %s" % (float(r["TotalDurationNs"]) / 1e3, r["Calls"], r["Name"][:90]))
PY
