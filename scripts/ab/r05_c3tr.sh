#!/bin/bash
# C3 kernel traces: the round-3 tree vs this tree (--pair-table 3), one box
set -o pipefail
cd "$(dirname "$0")/../.."
O=$PWD/gpurun_out/r05c3tr; mkdir -p $O
export TMPDIR=/tmp
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean --steps 40 --warmup 10 --epochs 0 --no-cpu-baseline --sampler-batches 0 --no-secondary-af"
(cd scripts/probe/r03tree && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r03 -o run --output-format csv -- \
  python3 bench.py $C3 > $O/r03.log 2>&1) || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cur -o run --output-format csv -- \
  python3 bench.py $C3 --pair-table 3 --no-secondary-exact --no-secondary-mt > $O/cur.log 2>&1
