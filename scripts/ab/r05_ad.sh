#!/bin/bash
# kernel trace of the GPU sampler alone (bench's sampler-only phase, C2)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ad; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --epochs 0 --no-cpu-baseline --no-interference-probe \
  --no-secondary-af --no-secondary-exact --no-secondary-mt --sampler-batches 32 > $O/trace.log 2>&1
