#!/bin/bash
# MT19937 mode: banded resolver — bit-exact tests, the --rng mt step, its trace
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05z; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py tests/test_fullsize.py -k "mt19937" > $O/tests.log 2>&1 || exit 1
A="--secondary --rng mt --steps 20 --warmup 5"
timeout -k 10 300 python -u bench.py $A > $O/mt.json 2> $O/mt.log || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 bench.py $A > $O/trace.log 2>&1
