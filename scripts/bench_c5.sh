#!/bin/bash
# BASELINE config 5 shapes on one GPU: papers100M-shaped (V = 111 M, E = 3.3 B, F = 128),
# GraphSAGE 3-layer 15/10/5, B = 1024: all-HBM, then the GS_SAMPLE_PD_CACHE form
# (features in pinned host memory with 30% cached in HBM + the NeutronOrch PD cache).
set -o pipefail
O=gpurun_out/c5_${1:-a}
mkdir -p $O
run() {
  local tag=$1; shift
  timeout -k 10 700 python -u bench.py --no-cpu-baseline --shape papers100m --layers 128-256-256-172 --fanout 15-10-5 --batch 1024 --weight mean --steps 20 --warmup 5 --epochs 0 --sampler-batches 8 "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); c=d['config']
print('$tag', round(d['ms_per_step'],4), 'ms/step', '%.3g edges/s' % d['value'], 'epoch-est', round(c['epoch_time_s'],1), 'sampler-only %.3g' % c['gpu_sampler_only']['value'], d['roofline'].get('kernel'), round(d['roofline'].get('frac') or 0, 3))"
}
run hbm
run pd_cache --cache-rate 0.3 --pd-cache --pd-rate 0.2 --pd-super-batch 4 --train-limit 40960
