#!/bin/bash
# A/B of the bottom aggregation alone (training stream, no overlap)
set -o pipefail
mkdir -p gpurun_out
for v in "--no-early-agg" "--no-early-agg --no-pipeline" ""; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $v > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { echo BENCH FAILED $v; tail -20 gpurun_out/bench_ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_ab.json'));print('$v', round(d['ms_per_step'],3),'ms', round(d['value']/1e6),'M edges/s', 'agg', round(d['roofline']['avg_launch_ms'],3), 'ms frac', round(d['roofline']['frac'],3))"
done
