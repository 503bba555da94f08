#!/bin/bash
# Headline bench A/B: bottom-layer order x GEMM arithmetic (and extra env for all).
set -o pipefail
O=gpurun_out/ab_tf_${1:-a}
mkdir -p $O
for cfg in "0 f32" "0 split3" "1 split3"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --transform-first $1 --gemm $2 --no-cpu-baseline --epochs 2 --sampler-batches 0 > $O/tf$1_$2.json 2> $O/tf$1_$2.err || { echo "bench $cfg failed"; tail -5 $O/tf$1_$2.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/tf$1_$2.json').read().strip().splitlines()[-1])
print('tf$1 $2', round(d['ms_per_step'],4), 'ms/step', {k:(round(v['avg_launch_ms']*1e3,1)) for k,v in d['roofline'].get('kernels',{}).items()})"
done
