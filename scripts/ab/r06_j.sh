#!/bin/bash
# (1) aggregation: XCD-aware block order (lib_aggxcd) vs the product order,
#     scripts/micro_agg.py interleaved; (2) the MT19937 tests with the forced
#     short first bounds (walks bounded by the generated words, positions
#     clamped)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06j; mkdir -p $O
export TMPDIR=/tmp
( for i in $(seq 1 40); do sleep 30; date >> $O/heartbeat.txt; done ) &
HB=$!
for r in 1 2; do
  for v in base aggxcd; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 200 python -u scripts/micro_agg.py --iters 30 > $O/agg_${v}_$r.json 2>> $O/agg.log || { kill $HB; exit 1; }
  done
done
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
    tests/test_fullsize.py tests/test_hip_kernels.py -k "mt19937 or mt_" > $O/tests.log 2>&1
rc=$?
kill $HB
exit $rc
