#!/bin/bash
# Round-4 batch H: the sampler-gate tests and its C2 A/B (0 / 1 / 2, twice).
set -o pipefail
O=gpurun_out/${1:-r04h}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gate or pipeline" > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
for r in 1 2; do
  for g in 0 1 2; do
    timeout -k 10 300 python -u bench.py $B --sampler-gate $g > $O/b_${g}_$r.json 2> $O/b_${g}_$r.err || { echo "bench gate $g failed"; tail -5 $O/b_${g}_$r.err; exit 1; }
    python3 - $O/b_${g}_$r.json $g <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = d["config"].get("training_stream_alone") or {}
print("gate", sys.argv[2], round(d["ms_per_step"], 4), "ms/step; alone", round(a.get("ms_per_step", 0), 4), {k: v.get("pipelined") for k, v in (a.get("kernel_avg_us") or {}).items()})
PY
  done
done
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mt19937 or fanout_above" > $O/mt_tests.log 2>&1 || { echo "mt tests failed"; tail -30 $O/mt_tests.log; exit 1; }
tail -1 $O/mt_tests.log
timeout -k 10 300 python -u bench.py --rng mt --steps 20 --warmup 3 $B --no-interference-probe > $O/mt.json 2> $O/mt.err || { echo "mt failed"; tail -5 $O/mt.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/mt.json').read().strip().splitlines()[-1]); print('MT', round(d['ms_per_step'],3), 'ms/step', '%.3g' % d['value'])"
