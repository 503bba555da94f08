#!/bin/bash
# MT parity tests and the --rng mt step with 192-dst chunks for the second layer
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ak; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py tests/test_fullsize.py -k "mt19937" > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --secondary --rng mt --steps 20 --warmup 5 > $O/mt.json 2> $O/mt.log
