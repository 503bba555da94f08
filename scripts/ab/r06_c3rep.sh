#!/bin/bash
# C3 repeated, product vs lib_nox3k interleaved (an outlier check)
set -o pipefail
O=gpurun_out/r06am; mkdir -p $O
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0"
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean"
for r in 1 2 3; do
  for v in base nox3k; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B $C3 --steps 40 --warmup 10 > $O/c3_${v}_$r.json 2>> $O/bench.log || exit 1
  done
done
