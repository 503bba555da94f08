#!/bin/bash
# Round-4 batch O: the MT window tables' register window, n + 4 / 6 / 8 / 12
# words (scripts/probe/lib_nw*, make variant VFLAGS=-DNTS_MT_NWX=k): MT parity
# tests and the --rng mt C2 bench for each.
set -o pipefail
O=gpurun_out/${1:-r04o}
mkdir -p $O
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 --rng mt --steps 10 --warmup 2 --no-interference-probe"
for v in nw4 nw6 product nw12 nw4 nw6 product nw12; do
  if [ $v = product ]; then L="NTS_NONE=0"; else L="NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so"; fi
  env $L timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mt19937" > $O/t_$v.log 2>&1 || { echo "tests $v failed"; tail -20 $O/t_$v.log; exit 1; }
  env $L timeout -k 10 300 python -u bench.py $B > $O/mt_$v.json 2> $O/mt_$v.err || { echo "bench $v failed"; tail -5 $O/mt_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/mt_$v.json').read().strip().splitlines()[-1]); print('$v MT C2', round(d['ms_per_step'],4))"
done
