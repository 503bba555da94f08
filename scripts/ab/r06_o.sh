#!/bin/bash
# k_x3_nn7 relu/dropout epilogue without scratch: GEMM tests, C3 / C4 benches, C3 trace
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1 || exit 1
bash scripts/bench_configs.sh r06o > $O/configs.txt 2>&1 || exit 1
bash scripts/prof_c3.sh r06c3c > $O/c3prof.txt 2>&1 || exit 1
