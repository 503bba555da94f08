#!/bin/bash
# A/B on one box: the library at HEAD (scripts/probe/lib_head) vs the working tree
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05q; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  NTS_HIP_LIB=scripts/probe/lib_head/libnts_hip.so timeout -k 10 60 \
      python -u scripts/micro_x3.py --iters 50 --tag head >> $O/micro.jsonl 2>&1 || exit 1
  timeout -k 10 60 python -u scripts/micro_x3.py --iters 50 --tag new >> $O/micro.jsonl 2>&1 || exit 1
done
