#!/bin/bash
# Pair-table (f16 two-piece) transform-first A/B: host parity tests, then the
# C2 bench aggregate-first vs transform-first with pair tables 0/1/2.
#   scripts/ab_h2.sh [tag]
set -o pipefail
TAG=${1:-h2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_host.py tests/test_gemm_h2.py -x -q --timeout 120 --timeout-method thread -k "forward_activations or training_step or transform_first or one_rank or h2" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B="--no-cpu-baseline --epochs 1 --sampler-batches 0 --steps 30 --warmup 5"
timeout -k 10 200 python -u bench.py $B --transform-first 0 > $O/af.json 2> $O/af.err || { tail -20 $O/af.err; exit 1; }
for pt in 0 1 2; do
  timeout -k 10 200 python -u bench.py $B --transform-first 1 --pair-table $pt > $O/tf$pt.json 2> $O/tf$pt.err || { tail -20 $O/tf$pt.err; exit 1; }
done
python - <<PY
import json
for f in ("af", "tf0", "tf1", "tf2"):
    d = json.loads(open("$O/%s.json" % f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 4), "ms/step", "%.4g" % d["value"], {k: (round(v["avg_launch_ms"]*1e3,1), round(v["frac"],3)) for k, v in d["roofline"].get("kernels", {}).items()})
PY
