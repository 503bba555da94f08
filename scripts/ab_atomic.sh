#!/bin/bash
# Graph-op backward: deterministic CSR gather (default) vs atomic CSC scatter
set -o pipefail
O=gpurun_out/ab_atomic_${1:-a}
mkdir -p $O
run() {
  local tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --sampler-batches 0 --epochs 1 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); c=d['config']
print('$tag', round(d['ms_per_step'],4), 'ms/step', 'issue', round(c['host_train_issue_s_per_step']*1e3,3), 'wait', round(c['host_sampler_wait_s_per_step']*1e3,3))"
}
run c2 
run c2_atomic --atomic-backward
run c3 --shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean --steps 40 --warmup 10
run c3_atomic --shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean --steps 40 --warmup 10 --atomic-backward
run c4 --shape products --layers 100-256-47 --fanout 25-10 --batch 1024 --steps 40 --warmup 10
run c4_atomic --shape products --layers 100-256-47 --fanout 25-10 --batch 1024 --steps 40 --warmup 10 --atomic-backward
