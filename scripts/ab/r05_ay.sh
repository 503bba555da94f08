#!/bin/bash
# fused output layer + loss alone: the K-split form (default, one 4-wave block
# per 16-row tile) vs the per-wave form (NTS_TOP_KSPLIT=0, one wave per tile)
# at the C2 and C3/C4 top-layer shapes and two between
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ay; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for s in "10000 128 41" "1024 256 47" "4096 256 47" "2500 128 41"; do
    set -- $s
    timeout -k 10 120 python -u scripts/micro_top.py --n $1 --K $2 --C $3 >> $O/ks1.jsonl 2>> $O/ks1.log || exit 1
    NTS_HIP_LIB=scripts/probe/lib_ks0/libnts_hip.so timeout -k 10 120 python -u scripts/micro_top.py \
        --n $1 --K $2 --C $3 >> $O/ks0.jsonl 2>> $O/ks0.log || exit 1
  done
done
