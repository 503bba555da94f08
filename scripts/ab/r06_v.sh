#!/bin/bash
# automatic sampler priority (normal for Philox, high for MT19937) vs the
# sampler stream always high (--sampler-high-priority): C2, C3, C4 interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06aa; mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0"
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean"
C4="--shape products --layers 100-256-47 --fanout 25-10 --batch 1024"
for r in 1 2; do
  for v in auto high; do
    if [ $v = auto ]; then X=; else X=--sampler-high-priority; fi
    timeout -k 10 200 python -u bench.py $B --steps 30 --warmup 5 $X > $O/c2_${v}_$r.json 2>> $O/bench.log || exit 1
    timeout -k 10 200 python -u bench.py $B $C3 --steps 40 --warmup 10 $X > $O/c3_${v}_$r.json 2>> $O/bench.log || exit 1
    timeout -k 10 200 python -u bench.py $B $C4 --steps 40 --warmup 10 $X > $O/c4_${v}_$r.json 2>> $O/bench.log || exit 1
  done
done
