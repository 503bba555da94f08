#!/bin/bash
# MT19937 word bound: the coupon-collector graphs, C3 3-layer MT, the existing MT tests
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py -k "mt19937" tests/test_fullsize.py::test_c3_mt19937_three_layers \
    tests/test_fullsize.py::test_c2_mt19937_reference_stream_full_batch > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --rng mt --steps 20 --warmup 5 --no-cpu-baseline \
    --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 > $O/mt.json 2> $O/mt.log
