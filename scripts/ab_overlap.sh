#!/bin/bash
# Sampler/training overlap variants at the headline config (aggregate-first).
set -o pipefail
O=gpurun_out/ab_overlap_${1:-a}
mkdir -p $O
run() {
  local tag=$1; shift
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --epochs 1 --sampler-batches 0 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print('$tag', round(d['ms_per_step'],4), 'ms/step', 'agg', round(d['roofline']['avg_launch_ms']*1e3,1))"
}
run base
run nopipe --no-pipeline
run early --early-agg
run cus16 --sampler-cus 16
run cus32 --sampler-cus 32
run noprio --no-priority
