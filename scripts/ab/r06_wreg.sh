#!/bin/bash
# k_x3_nn7 with the W image through registers (product) vs by LDS DMA with the
# counted wait (lib_wdma): the bit-exact gather tests 3x, then the C2 line
# interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06ap; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
      tests/test_gemm_split3.py tests/test_gemm_x3.py >> $O/tests.log 2>&1 || exit 1
done
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0"
for r in 1 2; do
  for v in base wdma; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B --steps 30 --warmup 5 > $O/c2_${v}_$r.json 2>> $O/bench.log || exit 1
  done
done
