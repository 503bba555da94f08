#!/bin/bash
# k_x3_nn7 W wait: vmcnt(8) (product) vs vmcnt(0) (lib_n7w0: every load
# drained at each step's wait — the one-tile form's race disappears with it):
# TN micro and the C2 line interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06an; mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0"
for r in 1 2; do
  for v in base n7w0; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 200 python -u scripts/micro_x3.py > $O/micro_${v}_$r.jsonl 2>> $O/micro.log || exit 1
    NTS_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B --steps 30 --warmup 5 > $O/c2_${v}_$r.json 2>> $O/bench.log || exit 1
  done
done
