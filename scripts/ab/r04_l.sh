#!/bin/bash
# Round-4 batch L: the pipelined sampler confined to n CUs with the training
# stream left on all 256 (--sampler-cus -n), against no masks; C2, twice each.
set -o pipefail
O=gpurun_out/${1:-r04l}
mkdir -p $O
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
for c in 0 -32 -64 -128 0 -32 -64 -128; do
  timeout -k 10 300 python -u bench.py $B --sampler-cus=$c > $O/b_$c.json 2> $O/b_$c.err || { echo "bench $c failed"; tail -5 $O/b_$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$c.json').read().strip().splitlines()[-1]); a=d['config'].get('training_stream_alone') or {}; print('cus $c C2', round(d['ms_per_step'],4), 'alone', round(a.get('ms_per_step',0),4), {k: v['pipelined'] for k, v in (a.get('kernel_avg_us') or {}).items()})"
done
