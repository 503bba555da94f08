#!/bin/bash
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
for cfg in "64 256" "32 256" "64 128" "32 128" "64 64" "16 256"; do
  set -- $cfg
  NTS_MT_CSZ_S=$1 NTS_MT_CSZ_B=$2 timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mt19937" > $O/t_$1_$2.log 2>&1 || { echo "tests $1 $2 failed"; tail -30 $O/t_$1_$2.log; exit 1; }
  NTS_MT_CSZ_S=$1 NTS_MT_CSZ_B=$2 timeout -k 10 300 python -u bench.py $B --rng mt --steps 10 --warmup 2 --no-interference-probe > $O/mt_$1_$2.json 2> $O/mt_$1_$2.err || { echo "bench failed"; tail -5 $O/mt_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/mt_$1_$2.json').read().strip().splitlines()[-1]); print('csz $1 $2 MT C2', round(d['ms_per_step'],4))"
done
