#!/bin/bash
# Round-4 batch P: --rng mt C2 with the stream priorities swapped
# (--training-priority) or both normal (--no-priority) against the default.
set -o pipefail
O=gpurun_out/${1:-r04p}
mkdir -p $O
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 --rng mt --steps 10 --warmup 2 --no-interference-probe"
for v in def tprio noprio def tprio noprio; do
  case $v in def) X="";; tprio) X="--training-priority";; noprio) X="--no-priority";; esac
  timeout -k 10 300 python -u bench.py $B $X > $O/mt_$v.json 2> $O/mt_$v.err || { echo "bench $v failed"; tail -5 $O/mt_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/mt_$v.json').read().strip().splitlines()[-1]); print('$v MT C2', round(d['ms_per_step'],4))"
done
