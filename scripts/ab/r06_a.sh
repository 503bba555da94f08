#!/bin/bash
# fp32-exact gathered GEMMs alone (scripts/micro_x3.py), interleaved on one box:
# the product build vs -fno-slp-vectorize (no v_pk_add_f32 in the splits),
# static s_setprio 1 for waves 4-7 (-DNTS_X3_PRIO), and both; then the C2 line
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06a; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in base noslp prio noslpprio; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 120 python -u scripts/micro_x3.py --iters 30 --tag $v >> $O/micro.jsonl 2>> $O/micro.log || exit 1
  done
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.log || exit 1
