#!/bin/bash
# the non-headline BASELINE configurations on the current build
set -o pipefail
O=gpurun_out/${1:-cfg}
mkdir -p $O
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --epochs 1"
$B --shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean --steps 40 --warmup 10 > $O/c3.json 2> $O/c3.err || { echo c3 failed; tail -5 $O/c3.err; exit 1; }
$B --shape products --layers 100-256-47 --batch 1024 --steps 40 --warmup 10 > $O/c4.json 2> $O/c4.err || { echo c4 failed; tail -5 $O/c4.err; exit 1; }
$B --model gat > $O/gat.json 2> $O/gat.err || { echo gat failed; tail -5 $O/gat.err; exit 1; }
python - <<PY
import json
for c in ("c3", "c4", "gat"):
    d = json.loads(open("$O/%s.json" % c).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(c, round(d["ms_per_step"], 4), "ms/step", "%.4g" % d["value"], "epoch %.4g s" % d["config"].get("epoch_time_s", 0),
          "sampler-only %.4g" % d["config"].get("gpu_sampler_only", {}).get("value", 0), r.get("kernel"), round(r.get("frac", 0), 3))
PY
