#!/bin/bash
# Round-4 GPU round trip: suite + smoke + bench (scripts/gpu_check.sh), then the
# wave-state PMC passes of the C2 bench kernels (scripts/pmc_stalls.sh).
set -o pipefail
T=${1:-r04}
bash scripts/gpu_check.sh $T || exit 1
bash scripts/pmc_stalls.sh $T > gpurun_out/$T/stalls.txt 2>&1 || { tail -5 gpurun_out/$T/stalls.txt; exit 1; }
cat gpurun_out/$T/stalls.txt
