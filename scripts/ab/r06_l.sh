#!/bin/bash
# MT19937 window tables: per-union-word distances (product) vs each lane's
# pairwise compares (lib_mtpair): MT tests, then the --rng mt step interleaved
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06l; mkdir -p $O
export TMPDIR=/tmp
( for i in $(seq 1 40); do sleep 30; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_fullsize.py tests/test_hip_kernels.py -k "mt19937 or mt_" > $O/tests.log 2>&1 || { kill $HB; exit 1; }
A="--rng mt --steps 20 --warmup 5 --no-secondary-af --no-secondary-exact --no-cpu-baseline --epochs 0 --sampler-batches 0 --no-interference-probe"
for r in 1 2; do
  for v in base mtpair; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 300 python -u bench.py $A > $O/mt_${v}_$r.json 2> $O/mt_${v}_$r.log || { kill $HB; exit 1; }
  done
done
kill $HB
