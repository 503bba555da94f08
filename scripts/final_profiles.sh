#!/bin/bash
# End-of-round evidence on the committed build: GPU suite + smoke + C2 bench
# (+ reference order), the C2 rocprofv3 trace and PMC passes, C3 / C4 traces.
#   scripts/final_profiles.sh <tag>
set -o pipefail
T=${1:-r03m}
bash scripts/gpu_check.sh $T || exit 1
bash profiles/collect.sh $T 20 || exit 1
bash scripts/prof_c3.sh c3_$T > gpurun_out/c3_$T.txt 2>&1 || exit 1
export TMPDIR=/tmp
O=gpurun_out/c4_$T
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 bench.py --shape products --layers 100-256-47 --fanout 25-10 --batch 1024 --steps 40 --warmup 5 --no-cpu-baseline --epochs 0 --sampler-batches 0 --no-secondary-af > $O/bench.json 2> $O/bench.err || exit 1
echo done
