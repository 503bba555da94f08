#!/bin/bash
# hop-1 Philox select (k_select_philox_g16) grid cap 4096 (default) vs 8192 /
# 16384 blocks: the sampler alone and the C2 step
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05as; mkdir -p $O
export TMPDIR=/tmp
A="--no-cpu-baseline --epochs 0 --no-secondary-af --no-secondary-exact --no-secondary-mt --sampler-batches 32"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/base_$r.json 2> $O/base_$r.log || exit 1
  for v in 8192 16384; do
    NTS_HIP_LIB=scripts/probe/lib_sel$v/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
        > $O/sel${v}_$r.json 2> $O/sel${v}_$r.log || exit 1
  done
done
