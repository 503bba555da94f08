#!/bin/bash
# CSR transpose as one high-digit radix pass + k_csr_bucket (product) vs the
# two-pass radix sort + k_csr_finalize (lib_csr2): sampler / full-size / host
# tests, then the C2 line interleaved (interference, sampler alone)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06p; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py tests/test_fullsize.py tests/test_host.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in base csr2; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
        --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 > $O/bench_${v}_$r.json 2>> $O/bench.log || exit 1
  done
done
