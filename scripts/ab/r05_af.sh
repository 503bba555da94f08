#!/bin/bash
# k_x3_nn: rounds with one tile left on half the MFMAs (NT = 1) vs every round on
# both tiles (-DNTS_X3_NO_NT1), same box
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 60 python -u scripts/micro_x3.py --iters 50 --tag nt1 >> $O/micro.jsonl 2>&1 || exit 1
  NTS_HIP_LIB=scripts/probe/lib_nont1/libnts_hip.so timeout -k 10 60 \
      python -u scripts/micro_x3.py --iters 50 --tag both >> $O/micro.jsonl 2>&1 || exit 1
done
