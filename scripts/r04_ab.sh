#!/bin/bash
# Round-4 A/B round trip for the opt-in kernels: the LDS-staged aggregation
# (NTS_AGG_LDS=1) and the four-stage NN (NTS_H2_NN4=1) — their tests, micro
# benchmarks of each against the default, short C2 benches, and the wave-state
# PMC passes of the default build.
set -o pipefail
T=${1:-r04ab}
O=gpurun_out/$T
mkdir -p $O
NTS_AGG_LDS=1 timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "spmm or csr or agg or capacity" > $O/agg_tests.log 2>&1 || { echo "agg tests failed"; tail -30 $O/agg_tests.log; exit 1; }
tail -1 $O/agg_tests.log
NTS_H2_NN4=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_h2.py -m gpu -x -q --timeout 120 --timeout-method thread -k "h2p_gemm_gather" > $O/nn4_tests.log 2>&1 || { echo "nn4 tests failed"; tail -30 $O/nn4_tests.log; exit 1; }
tail -1 $O/nn4_tests.log
for e in NTS_AGG_LDS=0 NTS_AGG_LDS=1; do
  env $e timeout -k 10 200 python -u scripts/micro_agg.py > $O/micro_agg_$e.json 2> $O/micro_agg_$e.err || { echo "micro_agg $e failed"; tail -5 $O/micro_agg_$e.err; exit 1; }
  echo "$e $(cat $O/micro_agg_$e.json)"
done
for e in NTS_H2_NN4=0 NTS_H2_NN4=1; do
  env $e timeout -k 10 200 python -u scripts/micro_bottom.py > $O/micro_bottom_$e.json 2> $O/micro_bottom_$e.err || { echo "micro_bottom $e failed"; tail -5 $O/micro_bottom_$e.err; exit 1; }
  echo "$e $(cat $O/micro_bottom_$e.json)"
done
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
for e in NTS_NONE=0 NTS_AGG_LDS=1 NTS_H2_NN4=0; do
  env $e timeout -k 10 300 python -u bench.py $B > $O/bench_$e.json 2> $O/bench_$e.err || { echo "bench $e failed"; tail -5 $O/bench_$e.err; exit 1; }
  python3 - $O/bench_$e.json "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = d["config"].get("training_stream_alone") or {}
print(sys.argv[2], round(d["ms_per_step"], 4), "ms/step; alone", round(a.get("ms_per_step", 0), 4),
      {k: (round(v["avg_launch_ms"] * 1e3, 1), round(v["frac"], 3)) for k, v in d["roofline"].get("kernels", {}).items()},
      a.get("kernel_avg_us"))
PY
done
NTS_AGG_LDS=1 bash scripts/pmc_stalls.sh $T > $O/stalls.txt 2>&1 || { tail -5 $O/stalls.txt; exit 1; }
grep -E "k_agg_lds|k_h2_nn4" $O/stalls.txt
