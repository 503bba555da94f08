#!/bin/bash
# C2 transform-first: NN v3 grid size A/B (blocks per column block)
set -o pipefail
O=gpurun_out/${1:-nb1}
mkdir -p $O
B="--no-cpu-baseline --epochs 1 --sampler-batches 0 --steps 40 --warmup 5"
for nb in 256 512 768 256; do
  NTS_H2_NN_BLOCKS=$nb timeout -k 10 200 python -u bench.py $B > $O/b$nb.json 2>> $O/err.log || exit 1
  python3 -c "import json; d=json.loads(open('$O/b$nb.json').read().strip().splitlines()[-1]); print('$nb', round(d['ms_per_step'],4), {k:round(v['avg_launch_ms']*1e3,1) for k,v in d['roofline']['kernels'].items()})"
done
