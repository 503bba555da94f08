#!/bin/bash
# k_x3_nnk (short dense reductions, whole W image in LDS): GEMM tests, the C3
# bottom-layer micro, C3 / C4 / C2 lines
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r06ad}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gemm_x3.py tests/test_gemm_split3.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/micro_c3gemm.py > $O/micro.jsonl 2> $O/micro.log || exit 1
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0"
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean"
C4="--shape products --layers 100-256-47 --fanout 25-10 --batch 1024"
for r in 1 2; do
  timeout -k 10 200 python -u bench.py $B $C3 --steps 40 --warmup 10 > $O/c3_$r.json 2>> $O/bench.log || exit 1
  timeout -k 10 200 python -u bench.py $B $C4 --steps 40 --warmup 10 > $O/c4_$r.json 2>> $O/bench.log || exit 1
done
timeout -k 10 200 python -u bench.py $B --steps 30 --warmup 5 > $O/c2.json 2>> $O/bench.log || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_host.py tests/test_fullsize.py > $O/tests2.log 2>&1 || exit 1
