#!/bin/bash
# sampler-alone kernel trace + the headline's kernel trace (stats) on the fp32 defaults
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/prof_sampler.sh r05i_samp --no-secondary-mt > gpurun_out/r05i_samp.txt 2>&1 || exit 1
bash profiles/collect.sh r05i 20 trace-only > gpurun_out/r05i_collect.txt 2>&1
