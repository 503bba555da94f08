#!/bin/bash
# Round-4 batch B: kernel + full-size parity tests, the sampler trace, a C2
# bench, the MT19937 bench under a kernel trace, and the C3 per-step trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2 or c3 or c4" > $O/full.log 2>&1 || { echo "fullsize tests failed"; tail -30 $O/full.log; exit 1; }
tail -1 $O/full.log
bash scripts/prof_sampler.sh $(basename $O)_samp > $O/samp.txt 2>&1 || { tail -5 $O/samp.txt; exit 1; }
head -14 $O/samp.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 8 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = d["config"].get("training_stream_alone") or {}
print("C2", round(d["ms_per_step"], 4), "ms/step; alone", round(a.get("ms_per_step", 0), 4), a.get("kernel_avg_us"), "sampler-only %.3g" % d["config"]["gpu_sampler_only"]["value"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mt -o run --output-format csv -- python3 bench.py --rng mt --steps 6 --warmup 2 --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 --no-interference-probe > $O/mt.json 2> $O/mt.err || { echo "mt failed"; tail -5 $O/mt.err; exit 1; }
python3 - $O <<'PY'
import csv, glob, json, sys
o = sys.argv[1]
d = json.loads(open(o + "/mt.json").read().strip().splitlines()[-1])
print("MT", round(d["ms_per_step"], 3), "ms/step")
f = glob.glob(o + "/mt/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]:
    print("  %-60s calls=%-4s avg_us=%.1f pct=%s" % (r["Name"].split("(")[0][-60:], r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"]))
PY
bash scripts/prof_c3.sh $(basename $O)_c3 > $O/c3.txt 2>&1 || { tail -5 $O/c3.txt; exit 1; }
head -30 $O/c3.txt
timeout -k 10 120 scripts/probe/stream_probe 10 > $O/stream.txt 2>&1 || { echo "probe failed"; tail -5 $O/stream.txt; exit 1; }
cat $O/stream.txt
