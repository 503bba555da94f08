#!/bin/bash
# k_x3_nn7 (W image by LDS DMA, 3 buffers): tests; probes 64 = every row id &
# 1023 (an L2-resident working set: is the A stream's cost the DRAM access
# pattern — 128 B of each of ~115 K rows per k-step?), 68 = that and no A
# loads, 4 = no A loads; lib_wreg = the W image staged through registers
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for d in 0 64 4 68; do
    NTS_HIP_LIB=scripts/probe/lib/libnts_hip.so NTS_X3_DIAG=$d timeout -k 10 120 python -u scripts/micro_x3.py --iters 30 --tag diag$d >> $O/micro.jsonl 2>> $O/micro.log || exit 1
  done
  NTS_HIP_LIB=scripts/probe/lib_wreg/libnts_hip.so timeout -k 10 120 python -u scripts/micro_x3.py --iters 30 --tag wreg >> $O/micro.jsonl 2>> $O/micro.log || exit 1
done
