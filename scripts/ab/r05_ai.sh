#!/bin/bash
# MT19937 window tables: the fallback walk's list in scratch (occupancy 8 / 6
# waves per SIMD for NMAX 10 / 25) vs in LDS (-DNTS_MT_LDS_LST: 7 / 4); MT
# parity tests first
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ai; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py tests/test_fullsize.py -k "mt19937" > $O/tests.log 2>&1 || exit 1
A="--secondary --rng mt --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/mt_scr_$r.json 2> $O/mt_scr_$r.log || exit 1
  NTS_HIP_LIB=scripts/probe/lib_ldslst/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
      > $O/mt_lds_$r.json 2> $O/mt_lds_$r.log || exit 1
done
