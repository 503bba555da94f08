#!/bin/bash
# full GPU suite on the fp32-exact defaults, then the default bench line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log
