#!/bin/bash
# MT19937 (reference-stream) mode: phased window tables — bit-exact tests, then
# the C2 --rng mt step with the phased library vs a one-phase build (same box)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py tests/test_fullsize.py -k "mt19937" > $O/tests.log 2>&1 || exit 1
A="--secondary --rng mt --steps 20 --warmup 5"
timeout -k 10 300 python -u bench.py $A > $O/mt_phased.json 2> $O/mt_phased.log || exit 1
NTS_HIP_LIB=scripts/probe/lib_ph1/libnts_hip.so timeout -k 10 300 python -u bench.py $A > $O/mt_ph1.json 2> $O/mt_ph1.log || exit 1
timeout -k 10 300 python -u bench.py $A > $O/mt_phased2.json 2> $O/mt_phased2.log
