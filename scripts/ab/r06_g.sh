#!/bin/bash
# the full GPU suite on the round-6 tree (k_x3_nn7 default), then the default
# bench line (secondaries included)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log || exit 1
