#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 python -u scripts/micro_x3.py --iters 50 --tag product > $O/micro.jsonl 2>&1 || exit 1
for D in 1 2 4 5 6 8 12 14; do
  NTS_HIP_LIB=scripts/probe/lib/libnts_hip.so NTS_X3_DIAG=$D timeout -k 10 60 \
      python -u scripts/micro_x3.py --iters 50 --tag diag$D >> $O/micro.jsonl 2>&1 || exit 1
done
