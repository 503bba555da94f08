#!/bin/bash
# MT19937 mode: resolver phases A/B (compile-time builds under scripts/probe/)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05x; mkdir -p $O
export TMPDIR=/tmp
A="--secondary --rng mt --steps 20 --warmup 5"
for r in 1 2; do
  for v in ph1 p2 p3 p4 p4b; do
    NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
        > $O/mt_${v}_$r.json 2> $O/mt_${v}_$r.log || exit 1
  done
done
