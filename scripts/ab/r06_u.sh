#!/bin/bash
# sampler scheduling, second batch (interleaved on one box): default,
# --training-priority, --no-priority, and each with the sampler confined to
# 32 / 64 CUs (--sampler-cus -N, training on all CUs)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06z; mkdir -p $O
export TMPDIR=/tmp
B="--steps 30 --warmup 5 --no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0"
for r in 1 2; do
  for v in default tp np tp32 np32 tp64 tp16; do
    case $v in
      default) X=;; tp) X=--training-priority;; np) X=--no-priority;;
      tp32) X="--training-priority --sampler-cus -32";; np32) X="--no-priority --sampler-cus -32";;
      tp64) X="--training-priority --sampler-cus -64";; tp16) X="--training-priority --sampler-cus -16";;
    esac
    timeout -k 10 200 python -u bench.py $B $X > $O/b_${v}_$r.json 2>> $O/bench.log || exit 1
  done
done
