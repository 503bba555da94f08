#!/bin/bash
# sampler-side GPU tests, then the default bench line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05v; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py tests/test_fullsize.py tests/test_host.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
