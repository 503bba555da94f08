#!/bin/bash
# Round-4 batch E: compile-time A/B builds (scripts/probe/lib_<v>) against the
# product build — kernel tests under each, the aggregation / pair-table micro
# benchmarks, and a C2 bench line each.
set -o pipefail
O=gpurun_out/${1:-r04e}
mkdir -p $O
VARS=${VARS:-"lpd16 nn3acc2"}
for v in $VARS; do
  L="NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so"
  env $L timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_gemm_h2.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -20 $O/tests_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $O/tests_$v.log)"
done
for v in product $VARS product $VARS; do
  if [ $v = product ]; then L="NTS_NONE=0"; else L="NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so"; fi
  env $L timeout -k 10 200 python -u scripts/micro_agg.py > $O/ma_$v.json 2> $O/ma_$v.err || { echo "micro_agg $v failed"; tail -5 $O/ma_$v.err; exit 1; }
  env $L timeout -k 10 200 python -u scripts/micro_bottom.py > $O/mb_$v.json 2> $O/mb_$v.err || { echo "micro_bottom $v failed"; tail -5 $O/mb_$v.err; exit 1; }
  python3 - $O/ma_$v.json $O/mb_$v.json $v <<'PY'
import json, sys
a = json.load(open(sys.argv[1])); b = json.load(open(sys.argv[2]))
print(sys.argv[3], "agg bottom", a["bottom"]["fwd_us"], a["bottom"]["bwd_us"], "hop0", a["hop0"]["fwd_us"], a["hop0"]["bwd_us"], "| nn", b["nn_us"], "tn", b["tn_us"])
PY
done
for v in product $VARS; do
  if [ $v = product ]; then L="NTS_NONE=0"; else L="NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so"; fi
  env $L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 1; }
  python3 - $O/bench_$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = d["config"].get("training_stream_alone") or {}
print(sys.argv[2], "C2", round(d["ms_per_step"], 4), "ms/step; alone", round(a.get("ms_per_step", 0), 4), a.get("kernel_avg_us"))
PY
done
