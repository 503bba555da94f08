#!/bin/bash
# the register gather's ceiling for 512-B rows of a 117 MB table; the library's
# bottom aggregation at the same size (micro_agg.py)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/probe/gather_probe 20 > $O/gather.jsonl 2>&1 &&
timeout -k 10 120 python -u scripts/micro_agg.py > $O/micro_agg.jsonl 2>&1
