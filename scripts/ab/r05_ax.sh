#!/bin/bash
# MT19937 window tables: waves past the window leave (default) vs whole
# blocks only (NTS_MT_BLOCK_EXIT), and the window half-width 4 (default) /
# 3.5 / 3 sigmas (a Delta outside its window is walked out serially by the
# resolver); the MT parity tests on the narrowest variant first
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ax; mkdir -p $O
export TMPDIR=/tmp
NTS_HIP_LIB=scripts/probe/lib_sig3/libnts_hip.so timeout -k 10 600 python -u -m pytest -x -q \
    --timeout 300 --timeout-method thread -m gpu tests -k "mt19937 or mt_" > $O/tests_sig3.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    -k "mt19937 or mt_" > $O/tests_base.log 2>&1 || exit 1
A="--secondary --rng mt --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/mt_base_$r.json 2> $O/mt_base_$r.log || exit 1
  for v in bexit sig35 sig3; do
    NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
        > $O/mt_${v}_$r.json 2> $O/mt_${v}_$r.log || exit 1
  done
done
