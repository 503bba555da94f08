#!/bin/bash
# MT19937 window tables: the wave min / max by DPP + readlane (default) vs
# __shfl_xor butterflies (lib_mtold, the previous source): MT parity tests,
# the --rng mt step interleaved, then the round's record
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05bc; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    -k "mt19937 or mt_" > $O/tests_mt.log 2>&1 || exit 1
A="--secondary --rng mt --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/mt_new_$r.json 2> $O/mt_new_$r.log || exit 1
  NTS_HIP_LIB=scripts/probe/lib_mtold/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
      > $O/mt_old_$r.json 2> $O/mt_old_$r.log || exit 1
done
bash scripts/ab/r05_final.sh
