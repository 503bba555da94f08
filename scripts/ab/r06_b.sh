#!/bin/bash
# k_x3_nn7 (round 6 NN: 4-wave blocks, 7 row tiles a wave, A to registers)
# vs k_x3_nn (lib_nnv1): bit-exactness tests, micro timings interleaved, C2 line
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in base nnv1; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 120 python -u scripts/micro_x3.py --iters 30 --tag $v >> $O/micro.jsonl 2>> $O/micro.log || exit 1
  done
done
timeout -k 10 300 python -u bench.py --no-secondary-mt --no-secondary-exact --no-secondary-af > $O/bench.json 2> $O/bench.log || exit 1
