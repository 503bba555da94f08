#!/bin/bash
# default bench line (two runs) on the current library
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ah; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 400 python -u bench.py > $O/bench_$r.json 2> $O/bench_$r.log || exit 1
done
