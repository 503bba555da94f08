#!/bin/bash
# Round-4 end evidence, part B (committed build): the C2 bench under a kernel
# trace and the PMC passes (profiles/collect.sh), then the C3 and C4 traces.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r04}
bash profiles/collect.sh $T 20 || exit 1
bash scripts/prof_c3.sh c3_$T > gpurun_out/c3_$T.txt 2>&1 || { tail -5 gpurun_out/c3_$T.txt; exit 1; }
head -30 gpurun_out/c3_$T.txt
O=gpurun_out/c4_$T
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 bench.py --shape products --layers 100-256-47 --fanout 25-10 --batch 1024 --steps 40 --warmup 5 --no-cpu-baseline --epochs 0 --sampler-batches 0 --no-secondary-af > $O/bench.json 2> $O/bench.err || exit 1
echo done
