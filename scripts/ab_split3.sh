#!/bin/bash
# split-bf16 GEMM kernels: v2 (default) vs v1 (NTS_S3_V1=1), parity tests + micro timings.
set -o pipefail
O=gpurun_out/ab_split3_${1:-a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_split3.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "split3 tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u scripts/micro_split3.py > $O/micro_v2.log 2>&1 && timeout -k 10 120 python -u scripts/probe_split3.py > $O/probe_v2.log 2>&1 || { echo "v2 micro failed"; tail $O/*.log; exit 1; }
NTS_S3_V1=1 timeout -k 10 120 python -u scripts/micro_split3.py > $O/micro_v1.log 2>&1 || exit 1
grep split3 $O/micro_v1.log $O/micro_v2.log $O/probe_v2.log
