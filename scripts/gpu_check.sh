#!/bin/bash
# One GPU round trip: parity suite, smoke, default bench, aggregate-first A/B.
#   scripts/gpu_check.sh [tag] [pytest -k expr]
set -o pipefail
TAG=${1:-chk}
K=${2:-}
O=gpurun_out/$TAG
mkdir -p $O
# heartbeat under gpurun_out/ (some full-size tests run minutes without
# printing; each test still has its own --timeout)
( while true; do date +%T >> $O/heartbeat.txt; sleep 50; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=12 > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
fi
grep -E "passed|failed|s call" $O/tests.log | head -16
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --transform-first 0 --no-cpu-baseline --epochs 1 --sampler-batches 0 > $O/bench_af.json 2> $O/bench_af.err || { echo "bench af failed"; tail -20 $O/bench_af.err; exit 1; }
python - <<PY
import json
for f in ("$O/bench.json", "$O/bench_af.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 4), "ms/step", "%.4g" % d["value"], d["roofline"].get("kernel"), {k: (round(v["avg_launch_ms"]*1e3,1), round(v["frac"],3)) for k, v in d["roofline"].get("kernels", {}).items()})
PY
echo ok
