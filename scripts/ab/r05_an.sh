#!/bin/bash
# MT19937 window tables: drawing dsts' unions in flight (NTS_MT_PF 1 / 2 / 3 /
# 4) by LDS DMA; MT parity tests on the default (3) first
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05an; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py tests/test_fullsize.py -k "mt19937" > $O/tests.log 2>&1 || exit 1
A="--secondary --rng mt --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/mt_pf3_$r.json 2> $O/mt_pf3_$r.log || exit 1
  for v in 1 2 4; do
    NTS_HIP_LIB=scripts/probe/lib_pf$v/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
        > $O/mt_pf${v}_$r.json 2> $O/mt_pf${v}_$r.log || exit 1
  done
done
