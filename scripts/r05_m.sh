#!/bin/bash
# C3 / C4 on the fp32 defaults (pair tables off) vs --pair-table 3 (round 4's
# defaults: the narrow layer's f16 pair split k_h2_nnd), two runs each, one box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05m; mkdir -p $O
run() {
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --sampler-batches 16 --no-secondary-mt "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); c=d['config']
print('$tag', round(d['ms_per_step'],4), 'ms/step', '%.4g edges/s' % d['value'], 'epoch', round(c['epoch_time_s'],4), 'sampler-only %.3g' % c['gpu_sampler_only']['value'], 'alone', round(c['training_stream_alone']['ms_per_step'],4))"
}
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean --steps 40 --warmup 10 --epochs 2"
C4="--shape products --layers 100-256-47 --fanout 25-10 --batch 1024 --steps 40 --warmup 10 --epochs 2"
for i in 1 2; do
  run c3_fp32_$i $C3 && run c3_pair_$i $C3 --pair-table 3 && run c4_fp32_$i $C4 && run c4_pair_$i $C4 --pair-table 3 || exit 1
done
