#!/bin/bash
# k_x3_nn7 with the relu/dropout epilogue on dense rows (C3 / C4 bottom NN):
# GEMM tests, host tests, then C3 / C4 benches
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06n; mkdir -p $O
export TMPDIR=/tmp
( for i in $(seq 1 40); do sleep 30; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py tests/test_host.py > $O/tests.log 2>&1 || { kill $HB; exit 1; }
bash scripts/bench_configs.sh r06n > $O/configs.txt 2>&1 || { kill $HB; exit 1; }
kill $HB
