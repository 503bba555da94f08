#!/bin/bash
# kernel trace of the C2 --rng mt step (the reference-stream secondary)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py --secondary --rng mt --steps 20 --warmup 5 > $O/trace.log 2>&1
