#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1
timeout -k 10 60 python -u scripts/micro_x3.py --iters 50 --tag product > $O/micro.jsonl 2>&1 || exit 1
for D in 1 4 5 14; do
  NTS_HIP_LIB=scripts/probe/lib/libnts_hip.so NTS_X3_DIAG=$D timeout -k 10 60 \
      python -u scripts/micro_x3.py --iters 50 --tag diag$D >> $O/micro.jsonl 2>&1 || exit 1
done
