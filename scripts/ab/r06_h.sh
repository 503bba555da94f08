#!/bin/bash
# MT19937 short-stream re-run (ABI 11): the MT tests, incl. the forced
# short first bounds at C2 size with three slots in flight
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_fullsize.py tests/test_hip_kernels.py -k "mt19937 or mt_" > $O/tests.log 2>&1 || exit 1
