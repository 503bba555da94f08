#!/bin/bash
# MT19937 chunk sizes with the higher-occupancy window tables: the second
# layer's (mid) and the seed layer's (small) dsts per chunk, compile-time
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05aj; mkdir -p $O
export TMPDIR=/tmp
A="--secondary --rng mt --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/mt_base_$r.json 2> $O/mt_base_$r.log || exit 1
  for v in m96 m192 s48 s24; do
    NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
        > $O/mt_${v}_$r.json 2> $O/mt_${v}_$r.log || exit 1
  done
done
