#!/bin/bash
# k_x3_nn32 (32x32x16 MFMA NN): GEMM tests, then A/B vs the 16x16x32 k_x3_nn
# (-DNTS_NO_X3_32 build) at C2 size, and probes
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ac; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1
for r in 1 2; do
  timeout -k 10 60 python -u scripts/micro_x3.py --iters 50 --tag nn32 >> $O/micro.jsonl 2>&1 || exit 1
  NTS_HIP_LIB=scripts/probe/lib_no32/libnts_hip.so timeout -k 10 60 \
      python -u scripts/micro_x3.py --iters 50 --tag nn16 >> $O/micro.jsonl 2>&1 || exit 1
done
for D in 1 4 5 14; do
  NTS_HIP_LIB=scripts/probe/lib/libnts_hip.so NTS_X3_DIAG=$D timeout -k 10 60 \
      python -u scripts/micro_x3.py --iters 50 --tag diag$D >> $O/micro.jsonl 2>&1 || exit 1
done
