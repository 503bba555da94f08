#!/bin/bash
# drained DMA waits in k_x3_nn (gathered NN below 32,768 rows) and
# k_gemm3_nn (dense K >= 256): the GEMM / host tests (the host's
# transform-first dropout test 3x), then C3 and C2 against lib_s3cnt
# (k_gemm3_nn's counted wait) interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06ao; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py tests/test_host.py > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
      tests/test_host.py -k "transform_first_trains" >> $O/tests_tf.log 2>&1 || exit 1
done
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0"
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean"
for r in 1 2; do
  for v in base s3cnt; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B $C3 --steps 40 --warmup 10 > $O/c3_${v}_$r.json 2>> $O/bench.log || exit 1
  done
done
timeout -k 10 200 python -u bench.py $B --steps 30 --warmup 5 > $O/c2.json 2>> $O/bench.log || exit 1
