#!/bin/bash
# Two ranks on the one GPU (gloo timing collectives, no all-reduce): the
# multi-rank control flow of bench.py --gpus 2 under torch.distributed.run
set -o pipefail
O=gpurun_out/${1:-dp1}
mkdir -p $O
NTS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline \
  --epochs 1 --sampler-batches 0 > $O/dp2.json 2> $O/dp2.err || { tail -30 $O/dp2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/dp2.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['config']['parallelism'], round(d['ms_per_step'],4), '%.4g' % d['value'], d['config']['bottom_layer'])"
