#!/bin/bash
# r05a: the fp32-exact transform-first path (no pair table) as the headline:
# live per-kernel times + a kernel trace of the same command
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --pair-table 0 --transform-first 1 --steps 20 --warmup 5 \
    --no-cpu-baseline --no-secondary-af --no-secondary-mt --epochs 0 --sampler-batches 0 \
    > $O/exact.json 2> $O/exact.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py \
    --pair-table 0 --transform-first 1 --steps 20 --warmup 3 --no-cpu-baseline \
    --no-secondary-af --no-secondary-mt --epochs 0 --sampler-batches 0 --no-interference-probe \
    > $O/prof.log 2>&1
