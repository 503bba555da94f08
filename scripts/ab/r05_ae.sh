#!/bin/bash
# k_x3_nn with the next step's split pinned in the current step (asm use) vs
# not (-DNTS_X3_NOPIN), same box; the MT ring wrap-around test
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ae; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 60 python -u scripts/micro_x3.py --iters 50 --tag pin >> $O/micro.jsonl 2>&1 || exit 1
  NTS_HIP_LIB=scripts/probe/lib_nopin/libnts_hip.so timeout -k 10 60 \
      python -u scripts/micro_x3.py --iters 50 --tag nopin >> $O/micro.jsonl 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread -m gpu \
    tests/test_fullsize.py -k "ring_wraps" > $O/wrap.log 2>&1
