#!/bin/bash
# sizes words published by each layer's last kernel into mapped host memory
# (no per-batch D2H copy): full GPU suite, then the sampler alone + C2 step
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05at; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > $O/tests.log 2>&1 || exit 1
A="--no-cpu-baseline --epochs 0 --no-secondary-af --no-secondary-exact --no-secondary-mt --sampler-batches 32"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/run_$r.json 2> $O/run_$r.log || exit 1
done
