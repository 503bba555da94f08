#!/bin/bash
# hop-1/hop-0 Philox select (k_select_philox_g16): the 16-lane group's
# duplicate scan by DPP row broadcasts (NTS_SEL_DPP_BCAST) vs __shfl
# (ds_bpermute): the sampler parity tests on the variant, then the sampler
# alone and the C2 step interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ba; mkdir -p $O
export TMPDIR=/tmp
NTS_HIP_LIB=scripts/probe/lib_seldpp/libnts_hip.so timeout -k 10 600 python -u -m pytest -x -q \
    --timeout 300 --timeout-method thread -m gpu tests/test_hip_kernels.py tests/test_fullsize.py \
    -k "sampler or philox or c2 or c3" > $O/tests_seldpp.log 2>&1 || exit 1
A="--no-cpu-baseline --epochs 0 --no-secondary-af --no-secondary-exact --no-secondary-mt --sampler-batches 32"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/base_$r.json 2> $O/base_$r.log || exit 1
  NTS_HIP_LIB=scripts/probe/lib_seldpp/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
      > $O/dpp_$r.json 2> $O/dpp_$r.log || exit 1
done
