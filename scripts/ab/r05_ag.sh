#!/bin/bash
# host issue time per sampled batch (NTS_HOST_PROFILE) in the sampler-only phase
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ag; mkdir -p $O
export TMPDIR=/tmp
NTS_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --epochs 0 --no-cpu-baseline \
  --no-interference-probe --no-secondary-af --no-secondary-exact --no-secondary-mt --sampler-batches 32 \
  > $O/bench.json 2> $O/host.log
