#!/bin/bash
# C2 bench: aggregate-first vs transform-first (pair tables 1 and 3)
set -o pipefail
TAG=${1:-h2j}
O=gpurun_out/$TAG
mkdir -p $O
B="--no-cpu-baseline --epochs 1 --sampler-batches 0 --steps 30 --warmup 5"
run() { local name=$1; shift; timeout -k 10 200 env "$@" > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }; }
run af python -u bench.py $B --transform-first 0
run tf1 python -u bench.py $B --transform-first 1 --pair-table 1
run tf3 python -u bench.py $B --transform-first 1 --pair-table 3
python - <<PY
import json
for f in ("af", "tf1", "tf3"):
    d = json.loads(open("$O/%s.json" % f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 4), "ms/step", "%.4g" % d["value"], {k: (round(v["avg_launch_ms"]*1e3,1), round(v["frac"],3)) for k, v in d["roofline"].get("kernels", {}).items()})
PY
