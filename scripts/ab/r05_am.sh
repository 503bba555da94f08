#!/bin/bash
# kernel trace of the C2 --rng mt step, training stream serialised (--no-pipeline)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05am; mkdir -p $O
export TMPDIR=/tmp
A="--secondary --rng mt --steps 20 --warmup 5 --no-pipeline"
timeout -k 10 300 python -u bench.py $A > $O/mt.json 2> $O/mt.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py $A > $O/trace.log 2>&1
