#!/bin/bash
# C3 / C4 with k_x3_nnk on the short dense bottom-layer NN (product) vs the
# fp32-input kernel (lib_nox3k), interleaved on one box; the micro of each
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r06ah}; mkdir -p $O
export TMPDIR=/tmp
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0"
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean"
C4="--shape products --layers 100-256-47 --fanout 25-10 --batch 1024"
for r in 1 2; do
  for v in base nox3k; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B $C3 --steps 40 --warmup 10 > $O/c3_${v}_$r.json 2>> $O/bench.log || exit 1
    NTS_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B $C4 --steps 40 --warmup 10 > $O/c4_${v}_$r.json 2>> $O/bench.log || exit 1
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_x3.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/micro_c3gemm.py > $O/micro.jsonl 2> $O/micro.log || exit 1
