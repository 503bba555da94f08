#!/bin/bash
# k_x3_nn7 with the W image staged through registers (all of W(g+1) loaded at
# step g's start: hipcc's waits for the A registers exact) vs the LDS-DMA W
# image (lib_wdma); timing probes of the new form; tests; the C2 line
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in base wdma; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 120 python -u scripts/micro_x3.py --iters 30 --tag $v >> $O/micro.jsonl 2>> $O/micro.log || exit 1
  done
  for d in 2 4 6 8 62; do
    NTS_HIP_LIB=scripts/probe/lib/libnts_hip.so NTS_X3_DIAG=$d timeout -k 10 120 python -u scripts/micro_x3.py --iters 30 --tag diag$d >> $O/micro.jsonl 2>> $O/micro.log || exit 1
  done
done
timeout -k 10 300 python -u bench.py --no-secondary-mt --no-secondary-exact --no-secondary-af > $O/bench.json 2> $O/bench.log || exit 1
