#!/bin/bash
# k_csr_bucket (16-wave blocks; dst ids / weights as radix payloads): sampler tests, the sampler-only trace, C2 line
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r06r}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py tests/test_fullsize.py -k "sampler or c2_reddit or c3_products or c4 or csr" > $O/tests.log 2>&1 || exit 1
bash scripts/prof_sampler.sh ${1:-r06r}/samp --no-secondary-mt > $O/samp.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
    --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 > $O/bench.json 2>> $O/bench.log || exit 1
