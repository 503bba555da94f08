#!/bin/bash
# the pipelined sampler's scheduling against the training stream, interleaved
# on one box (round-6 sampler): default (sampler stream high priority),
# --no-priority, --training-priority, --sampler-gate 1, --sampler-cus -32
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06y; mkdir -p $O
export TMPDIR=/tmp
B="--steps 30 --warmup 5 --no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0"
for r in 1 2; do
  for v in default no-priority training-priority gate1 cus32; do
    case $v in
      default) X=;; no-priority) X=--no-priority;; training-priority) X=--training-priority;;
      gate1) X="--sampler-gate 1";; cus32) X="--sampler-cus -32";;
    esac
    timeout -k 10 200 python -u bench.py $B $X > $O/b_${v}_$r.json 2>> $O/bench.log || exit 1
  done
done
