#!/bin/bash
# Round-4 batch M: the MT19937 chunked resolver with 64-dst chunks for layers
# of up to 32 K dsts (the C2 seed layer: 157 chunks instead of 40) — the MT
# parity tests (Cora, every layer chunked; C2 full batch), then the --rng mt
# C2 bench twice.
set -o pipefail
O=gpurun_out/${1:-r04m}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mt19937" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $B --rng mt --steps 10 --warmup 2 --no-interference-probe > $O/mt_$i.json 2> $O/mt_$i.err || { echo "bench mt failed"; tail -5 $O/mt_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/mt_$i.json').read().strip().splitlines()[-1]); print('MT C2', round(d['ms_per_step'],4), '%.4g' % d['value'])"
done
