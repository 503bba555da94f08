#!/bin/bash
# two ranks sharing the box's one GPU (the shared-GPU DP rehearsal: gloo
# all-reduce through host copies) on the final library
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05ar; mkdir -p $O
export TMPDIR=/tmp
NTS_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 > $O/dp2.json 2> $O/dp2.log
