#!/bin/bash
# sampler interference: the sampler's stream on 16 / 32 CUs and the training
# stream on the other 240 / 224, the fp32-exact GEMM grids sized to match
# (-DNTS_X3_CUS), against the default (both streams on all 256 CUs)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ap; mkdir -p $O
export TMPDIR=/tmp
A="--no-cpu-baseline --sampler-batches 0 --epochs 0 --no-secondary-af --no-secondary-exact --no-secondary-mt"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A > $O/base_$r.json 2> $O/base_$r.log || exit 1
  NTS_HIP_LIB=scripts/probe/lib_cus240/libnts_hip.so timeout -k 10 300 python -u bench.py $A --sampler-cus 16 \
      > $O/c240_$r.json 2> $O/c240_$r.log || exit 1
  NTS_HIP_LIB=scripts/probe/lib_cus224/libnts_hip.so timeout -k 10 300 python -u bench.py $A --sampler-cus 32 \
      > $O/c224_$r.json 2> $O/c224_$r.log || exit 1
done
