#!/bin/bash
# C3 / C4 on the round-6 tree, then a C3 kernel trace (per-step breakdown)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
bash scripts/bench_configs.sh r06 > gpurun_out/configs_r06.txt 2>&1 || exit 1
bash scripts/prof_c3.sh r06c3 > gpurun_out/r06c3_prof.txt 2>&1 || exit 1
