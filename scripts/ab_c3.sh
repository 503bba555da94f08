#!/bin/bash
set -o pipefail
O=gpurun_out/ab_c3_${1:-a}
mkdir -p $O
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --sampler-batches 0 --epochs 1 --shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean --steps 40 --warmup 10 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); c=d['config']
print('$tag', round(d['ms_per_step'],4), 'ms/step', 'issue', round(c['host_train_issue_s_per_step']*1e3,3), 'wait', round(c['host_sampler_wait_s_per_step']*1e3,3))"
}
run split3
run f32 --gemm f32
NTS_DIAG_REUSE_SAMPLE=1 run reuse_split3 --epochs 0
run nopipe --no-pipeline
