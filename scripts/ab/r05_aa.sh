#!/bin/bash
# MT19937 mode: the sampler stream beside the training stream vs serialised
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05aa; mkdir -p $O
export TMPDIR=/tmp
A="--secondary --rng mt --steps 20 --warmup 5"
for v in "pipe:" "nopipe:--no-pipeline" "gate1:--sampler-gate 1" "gate2:--sampler-gate 2" "nopri:--no-priority"; do
  n=${v%%:*}; f=${v#*:}
  timeout -k 10 300 python -u bench.py $A $f > $O/mt_$n.json 2> $O/mt_$n.log || exit 1
done
