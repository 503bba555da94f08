#!/bin/bash
# Profile the headline bench on the GPU box (run from the repo root):
#   kernel trace + stats, then two separate PMC passes (FETCH_SIZE, WRITE_SIZE)
#   profiles/collect.sh <tag> <steps> [trace-only] [extra bench flags...]
# Output: gpurun_out/prof_<tag>/... ; summarise with profiles/summarize.py
set -e
TAG=${1:-r01}
STEPS=${2:-10}
MODE=${3:-all}
if [ $# -ge 3 ]; then shift 3; else shift $#; fi
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0 "$@" > $OUT/trace.log 2>&1
[ "$MODE" = "trace-only" ] && { echo done; exit 0; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/fetch -o run --output-format csv -- \
  python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0 "$@" > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/write -o run --output-format csv -- \
  python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0 "$@" > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT/hit -o run --output-format csv -- \
  python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0 "$@" > $OUT/hit.log 2>&1
# MFMA pipe and wave-state counters (one SQ/GRBM group)
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace -d $OUT/sq -o run --output-format csv -- \
  python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-secondary-af --no-secondary-exact --no-secondary-mt --epochs 0 --sampler-batches 0 "$@" > $OUT/sq.log 2>&1
echo done
