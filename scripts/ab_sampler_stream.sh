#!/bin/bash
# C2 transform-first: sampler stream priority / CU-mask A/B
set -o pipefail
O=gpurun_out/${1:-ss1}
mkdir -p $O
B="--no-cpu-baseline --epochs 1 --sampler-batches 0 --steps 40 --warmup 5"
run() { local name=$1; shift; echo "== $name" >> $O/err.log; timeout -k 10 200 python -u bench.py $B "$@" > $O/$name.json 2>> $O/err.log || exit 1; }
run base
run noprio --no-priority
run cus32 --sampler-cus 32
run cus64 --sampler-cus 64
run base2
for f in base noprio cus32 cus64 base2; do
  python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],4), {k:round(v['avg_launch_ms']*1e3,1) for k,v in d['roofline']['kernels'].items()})"
done
