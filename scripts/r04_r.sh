#!/bin/bash
# --rng mt C2 at 10 and 40 timed steps: does a longer run (the word ring
# wrapping) cost per step?
set -o pipefail
O=gpurun_out/${1:-r04r}
mkdir -p $O
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0 --rng mt --no-interference-probe"
for s in 10 40; do
  timeout -k 10 300 python -u bench.py $B --steps $s --warmup 2 > $O/mt_$s.json 2> $O/mt_$s.err || { echo "bench $s failed"; tail -5 $O/mt_$s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/mt_$s.json').read().strip().splitlines()[-1]); print('steps $s MT C2', round(d['ms_per_step'],4))"
done
