#!/bin/bash
# Training stream alone (NTS_DIAG_REUSE_SAMPLE=1: one sampled batch reused; diagnostic only)
set -o pipefail
O=gpurun_out/ab_reuse_${1:-a}
mkdir -p $O
for tf in 0 1; do
  NTS_DIAG_REUSE_SAMPLE=1 timeout -k 10 200 python -u bench.py --transform-first $tf --gemm split3 --no-cpu-baseline --epochs 0 --sampler-batches 0 > $O/tf$tf.json 2> $O/tf$tf.err || { echo "bench tf$tf failed"; tail -5 $O/tf$tf.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/tf$tf.json').read().strip().splitlines()[-1])
print('reuse tf$tf', round(d['ms_per_step'],4), 'ms/step', {k:(round(v['avg_launch_ms']*1e3,1)) for k,v in d['roofline'].get('kernels',{}).items()})"
done
