#!/bin/bash
# fused output layer: the label / gradient loads first, DPP group reductions,
# each wave finishing its quarter of the tile — its tests, phase times
# (NTS_TOP_TIMING probe build) and time per call, then the round's record
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05az; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py -k "xent" > $O/tests_split.log 2>&1 || exit 1
NTS_HIP_LIB=scripts/probe/lib_toptime/libnts_hip.so timeout -k 10 120 python -u scripts/micro_top.py \
    --iters 5 > $O/c2d.txt 2>&1 || exit 1
timeout -k 10 120 python -u scripts/micro_top.py > $O/split_c2.json 2>&1 || exit 1
timeout -k 10 120 python -u scripts/micro_top.py --n 1024 --K 256 --C 47 > $O/split_c3.json 2>&1 || exit 1
bash scripts/ab/r05_final.sh
