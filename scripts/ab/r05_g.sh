#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 60 python -u scripts/micro_x3.py --iters 50 --tag product > $O/micro.jsonl 2>&1 || exit 1
NTS_HIP_LIB=scripts/probe/lib_nox3/libnts_hip.so timeout -k 10 60 \
    python -u scripts/micro_x3.py --iters 50 --tag nox3 >> $O/micro.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --pair-table 0 --transform-first 1 --steps 20 --warmup 5 \
    --no-cpu-baseline --no-secondary-af --no-secondary-mt --epochs 0 --sampler-batches 0 \
    > $O/exact.json 2> $O/exact.log
