#!/bin/bash
# post-mask CSR gather (hop-0 backward) with a capped grid — several rows per
# lane group (NTS_AGG_PM_GRID 2048 / 4096 / 8192) against one row per group:
# its parity tests on each variant, micro_agg, then the C2 step
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05au; mkdir -p $O
export TMPDIR=/tmp
for v in 2048 4096 8192; do
  NTS_HIP_LIB=scripts/probe/lib_pm$v/libnts_hip.so timeout -k 10 300 python -u -m pytest -x -q \
      --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py -k "postmask or csr_bwd" \
      > $O/tests_pm$v.log 2>&1 || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python -u scripts/micro_agg.py > $O/agg_base_$r.json 2> $O/agg_base_$r.log || exit 1
  for v in 2048 4096 8192; do
    NTS_HIP_LIB=scripts/probe/lib_pm$v/libnts_hip.so timeout -k 10 200 python -u scripts/micro_agg.py \
        > $O/agg_pm${v}_$r.json 2> $O/agg_pm${v}_$r.log || exit 1
  done
done
A="--no-cpu-baseline --epochs 0 --no-secondary-af --no-secondary-exact --no-secondary-mt --sampler-batches 0"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/base_$r.json 2> $O/base_$r.log || exit 1
  for v in 4096 8192; do
    NTS_HIP_LIB=scripts/probe/lib_pm$v/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
        > $O/pm${v}_$r.json 2> $O/pm${v}_$r.log || exit 1
  done
done
