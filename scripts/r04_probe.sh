#!/bin/bash
# Streaming probe of the pair table's sorted sweep (scripts/probe/stream_probe.hip,
# built in-tree beforehand) and the two pair-table GEMMs alone.
set -o pipefail
O=gpurun_out/${1:-r04probe}
mkdir -p $O
timeout -k 10 120 scripts/probe/stream_probe 10 > $O/stream.txt 2>&1 || { echo "probe failed"; tail -5 $O/stream.txt; exit 1; }
cat $O/stream.txt
timeout -k 10 200 python -u scripts/micro_bottom.py > $O/micro_bottom.json 2> $O/micro_bottom.err || { echo "micro_bottom failed"; tail -5 $O/micro_bottom.err; exit 1; }
cat $O/micro_bottom.json
timeout -k 10 200 python -u scripts/micro_agg.py > $O/micro_agg.json 2> $O/micro_agg.err || { echo "micro_agg failed"; tail -5 $O/micro_agg.err; exit 1; }
cat $O/micro_agg.json
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "spmm or csr or agg" > $O/agg_tests.log 2>&1 || { echo "agg tests failed"; tail -30 $O/agg_tests.log; exit 1; }
tail -1 $O/agg_tests.log
bash scripts/bench_configs.sh r04 || exit 1
