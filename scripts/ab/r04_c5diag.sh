#!/bin/bash
# The C5 full-size test (hung in train_batch with the single-pass scans; the
# scan state's zeroing raced the first look-back kernel), then the full-size
# suite.  NTS_LAUNCH_TRACE=1 in the environment traces every launch.
set -o pipefail
T=${1:-r04c5}
O=gpurun_out/$T
mkdir -p $O
( while true; do date +%T >> $O/heartbeat.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u -m pytest tests/test_fullsize.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k c5_papers > $O/c5.log 2>&1 || { echo "c5 failed"; grep -v "^  File\|^    " $O/c5.log | tail -30; exit 1; }
grep -E "passed|failed" $O/c5.log
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread --durations=8 > $O/full.log 2>&1 || { echo "fullsize failed"; grep -v "^  File\|^    " $O/full.log | tail -30; exit 1; }
grep -E "passed|failed|s call" $O/full.log
