#!/bin/bash
# the gather's row ids / weights by v_readlane (the then default; not kept) vs __shfl (lib_aggold,
# the previous source): the aggregation kernels alone and the C2 step
# interleaved, then the round's record (full GPU suite first)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05bd; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py -k "spmm or gather or csr or csc" > $O/tests_agg.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u scripts/micro_agg.py > $O/agg_new_$r.json 2> $O/agg_new_$r.log || exit 1
  NTS_HIP_LIB=scripts/probe/lib_aggold/libnts_hip.so timeout -k 10 200 python -u scripts/micro_agg.py \
      > $O/agg_old_$r.json 2> $O/agg_old_$r.log || exit 1
done
A="--no-cpu-baseline --epochs 0 --no-secondary-af --no-secondary-exact --no-secondary-mt --sampler-batches 0"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/new_$r.json 2> $O/new_$r.log || exit 1
  NTS_HIP_LIB=scripts/probe/lib_aggold/libnts_hip.so timeout -k 10 300 python -u bench.py $A \
      > $O/old_$r.json 2> $O/old_$r.log || exit 1
done
bash scripts/ab/r05_final.sh
