#!/bin/bash
# Round-4 batch F: kernel + full-size parity tests (MT19937 stream ring), the
# MT bench under a kernel trace, C2 bench, and the 16-lane aggregation A/B
# (scripts/probe/lib_lpd16).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04f}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2 or c3 or c4" > $O/full.log 2>&1 || { echo "fullsize tests failed"; tail -30 $O/full.log; exit 1; }
tail -1 $O/full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mt -o run --output-format csv -- python3 bench.py --rng mt --steps 6 --warmup 2 --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 --no-interference-probe > $O/mt.json 2> $O/mt.err || { echo "mt failed"; tail -5 $O/mt.err; exit 1; }
python3 - $O <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
d = json.loads(open(f"{o}/mt.json").read().strip().splitlines()[-1])
print("MT", round(d["ms_per_step"], 3), "ms/step")
f = glob.glob(f"{o}/mt/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print("  %-60s calls=%-4s avg_us=%.1f pct=%s" % (r["Name"].split("(")[0][-60:], r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"]))
PY
timeout -k 10 300 python -u bench.py --rng mt --steps 10 --warmup 3 --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 --no-interference-probe > $O/mt_plain.json 2> $O/mt_plain.err || { echo "mt plain failed"; tail -5 $O/mt_plain.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/mt_plain.json').read().strip().splitlines()[-1]); print('MT (no profiler)', round(d['ms_per_step'],3), 'ms/step', '%.3g' % d['value'])"
VARS=lpd16 bash scripts/r04_e.sh $(basename $O)_e || exit 1
