#!/bin/bash
# C3 / C4 regression A/B on one box: the round-3 tree (dec37f0, its own
# defaults: f16 pair tables) vs this tree with --pair-table 3 (the same
# numerics) and with its fp32-exact defaults; interleaved, two rounds
set -o pipefail
cd "$(dirname "$0")/../.."
O=$PWD/gpurun_out/r05c34b; mkdir -p $O
export TMPDIR=/tmp
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean --steps 40 --warmup 10 --epochs 2"
C4="--shape products --layers 100-256-47 --fanout 25-10 --batch 1024 --steps 40 --warmup 10 --epochs 2"
NEW="--no-cpu-baseline --sampler-batches 16 --no-secondary-af --no-secondary-exact --no-secondary-mt"
OLD="--no-cpu-baseline --sampler-batches 16 --no-secondary-af"
for i in 1 2; do
  for c in C3 C4; do
    args=${!c}
    (cd scripts/probe/r03tree && timeout -k 10 400 python -u bench.py $OLD $args > $O/${c}_r03_$i.json 2> $O/${c}_r03_$i.err) || exit 1
    timeout -k 10 400 python -u bench.py $NEW $args --pair-table 3 > $O/${c}_pair_$i.json 2> $O/${c}_pair_$i.err || exit 1
    timeout -k 10 400 python -u bench.py $NEW $args > $O/${c}_fp32_$i.json 2> $O/${c}_fp32_$i.err || exit 1
  done
done
timeout -k 10 400 python -u bench.py > $O/c2.json 2> $O/c2.err
