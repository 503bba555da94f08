#!/bin/bash
# the MT19937 tests (forced short first bounds included)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06k; mkdir -p $O
export TMPDIR=/tmp
( for i in $(seq 1 40); do sleep 30; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
    tests/test_fullsize.py tests/test_hip_kernels.py -k "mt19937 or mt_" > $O/tests.log 2>&1
rc=$?
kill $HB
exit $rc
