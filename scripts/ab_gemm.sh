#!/bin/bash
# A/B of the bottom-layer order x GEMM arithmetic at the headline config.
set -o pipefail
O=gpurun_out/ab_gemm_${1:-a}
mkdir -p $O
for tf in 0 1; do for gm in f32 split3; do
  timeout -k 10 200 python -u bench.py --transform-first $tf --gemm $gm --no-cpu-baseline --epochs 1 --sampler-batches 0 > $O/tf${tf}_${gm}.json 2> $O/tf${tf}_${gm}.err || { echo "bench tf$tf $gm failed"; tail -5 $O/tf${tf}_${gm}.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/tf${tf}_${gm}.json').read().strip().splitlines()[-1])
print('tf$tf $gm', round(d['ms_per_step'],4), 'ms/step', {k:(round(v['avg_launch_ms']*1e3,1)) for k,v in d['roofline'].get('kernels',{}).items()})"
done; done
