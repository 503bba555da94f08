#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py > $O/tests.log 2>&1 &&
timeout -k 10 120 python -u scripts/micro_x3.py > $O/micro.jsonl 2>&1
