#!/bin/bash
# k_x3_tn with the drained step wait + the masked one-tile form on C3 / C4's
# bottom weight gradient: GEMM / host / full-size tests, the race repro x40,
# then C3 / C4 interleaved against lib_nox3k (the fp32-input kernels)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06al; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py tests/test_host.py tests/test_fullsize.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/dbg_tn.py 40 > $O/dbg.txt 2>&1 || exit 1
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
timeout -k 10 200 python -u bench.py $B --steps 30 --warmup 5 > $O/c2.json 2>> $O/bench.log || exit 1
