#!/bin/bash
# CSR transpose (radix pass with payloads, 1,024-item tiles; k_csr_bucket): sampler tests, the sampler-only trace, C2 line
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-r06r}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu ${TESTS_K:+-k "$TESTS_K"} \
    tests/test_hip_kernels.py tests/test_fullsize.py tests/test_host.py > $O/tests.log 2>&1 || exit 1
bash scripts/prof_sampler.sh ${1:-r06r}/samp --no-secondary-mt > $O/samp.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
    --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 > $O/bench.json 2>> $O/bench.log || exit 1
