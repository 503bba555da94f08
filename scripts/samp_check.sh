#!/bin/bash
# sampler change: parity suite + default bench (gpu_check), the sampler alone
# under rocprofv3, and the C3 / C4 configurations
set -o pipefail
T=${1:-sc}
bash scripts/gpu_check.sh $T && bash scripts/prof_sampler.sh ${T}_prof || exit 1
O=gpurun_out/$T
timeout -k 10 300 python -u bench.py --no-cpu-baseline --epochs 1 --shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean --steps 40 --warmup 10 > $O/c3.json 2> $O/c3.err || { echo c3 failed; tail -5 $O/c3.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --epochs 1 --shape products --layers 100-256-47 --batch 1024 --steps 40 --warmup 10 > $O/c4.json 2> $O/c4.err || { echo c4 failed; tail -5 $O/c4.err; exit 1; }
python - <<PY
import json
for c in ("c3", "c4"):
    d = json.loads(open("$O/%s.json" % c).read().strip().splitlines()[-1])
    print(c, round(d["ms_per_step"], 4), "ms/step", "%.4g" % d["value"], "sampler-only %.4g" % d["config"].get("gpu_sampler_only", {}).get("value", 0))
PY
