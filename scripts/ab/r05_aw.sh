#!/bin/bash
# the bottom activation's keep mask as bits (16 B a row) for the fused hop-0
# backward, against the float mask rows (NTS_TF_MASK_FLOAT=1): the full GPU
# suite, then the C2 step interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05aw; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > $O/tests.log 2>&1 || exit 1
A="--no-cpu-baseline --epochs 0 --no-secondary-af --no-secondary-exact --no-secondary-mt --sampler-batches 0"
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py $A > $O/bits_$r.json 2> $O/bits_$r.log || exit 1
  NTS_TF_MASK_FLOAT=1 timeout -k 10 300 python -u bench.py $A > $O/float_$r.json 2> $O/float_$r.log || exit 1
done
