#!/bin/bash
# default bench line, then a kernel trace of the headline steps
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log || exit 1
bash profiles/collect.sh r05t 20 trace-only
