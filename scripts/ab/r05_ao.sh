#!/bin/bash
# the other BASELINE configurations on the current library: C3, C4, GAT, C5
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
bash scripts/bench_configs.sh r05 > gpurun_out/configs_r05.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --model gat --sampler-batches 8 \
    --no-secondary-af --no-secondary-exact --no-secondary-mt > gpurun_out/configs_r05/gat.json 2> gpurun_out/configs_r05/gat.err || exit 1
bash scripts/bench_c5.sh r05 > gpurun_out/c5_r05.txt 2>&1
