#!/bin/bash
# (epochs 0: the reuse diagnostic never ends a pass)
# Training stream alone (NTS_DIAG_REUSE_SAMPLE=1, diagnostic) vs the pipelined step
set -o pipefail
O=gpurun_out/${1:-diag1}
mkdir -p $O
B="--no-cpu-baseline --epochs 0 --sampler-batches 0 --steps 30 --warmup 5"
timeout -k 10 200 python -u bench.py $B > $O/tf.json 2>>$O/err.log &&
NTS_DIAG_REUSE_SAMPLE=1 timeout -k 10 200 python -u bench.py $B > $O/tf_reuse.json 2>>$O/err.log &&
NTS_DIAG_REUSE_SAMPLE=1 timeout -k 10 200 python -u bench.py $B --transform-first 0 > $O/af_reuse.json 2>>$O/err.log || exit 1
for f in tf tf_reuse af_reuse; do
  python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],4), {k:round(v['avg_launch_ms']*1e3,1) for k,v in d['roofline']['kernels'].items()})"
done
