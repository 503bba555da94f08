#!/bin/bash
# GPU suite, then the headline bench and C3 with the two-kernel scans
# (NTS_SCAN1=0) and with the single-pass look-back scans (the default).
#   scripts/ab_scan.sh [tag]
set -o pipefail
O=gpurun_out/${1:-scan}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean"
for s in 0 1; do
  NTS_SCAN1=$s timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --epochs 1 > $O/c2_s$s.json 2> $O/c2_s$s.err || { echo "c2 failed"; tail -20 $O/c2_s$s.err; exit 1; }
  NTS_SCAN1=$s timeout -k 10 300 python -u bench.py $C3 --steps 40 --warmup 10 --no-cpu-baseline --no-secondary-af --epochs 0 > $O/c3_s$s.json 2> $O/c3_s$s.err || { echo "c3 failed"; tail -20 $O/c3_s$s.err; exit 1; }
done
python3 - $O <<'PY'
import json, sys
for t in ("c2_s0", "c2_s1", "c3_s0", "c3_s1"):
    d = json.loads(open(f"{sys.argv[1]}/{t}.json").read().strip().splitlines()[-1])
    so = (d["config"].get("gpu_sampler_only") or {}).get("value")
    print(t, round(d["ms_per_step"], 4), "ms/step", "%.4g" % d["value"], "sampler-only", so and "%.4g" % so,
          {k: (round(v["avg_launch_ms"] * 1e3, 1), round(v["frac"], 3)) for k, v in d["roofline"].get("kernels", {}).items()})
PY
