#!/bin/bash
# Round-4 GPU round trip: aggregation kernel tests first (fast fail), suite +
# smoke + bench (scripts/gpu_check.sh), the four-stage NN's tests and an A/B
# bench (NTS_H2_NN4=1), an A/B bench of the register gather (NTS_AGG_LDS=0),
# then the wave-state PMC passes (scripts/pmc_stalls.sh).
set -o pipefail
T=${1:-r04}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "spmm or csr or agg" > $O/agg_tests.log 2>&1 || { echo "agg tests failed"; tail -30 $O/agg_tests.log; exit 1; }
tail -2 $O/agg_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=12 > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed|s call" $O/tests.log | head -16
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
NTS_H2_NN4=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_h2.py -m gpu -x -q --timeout 120 --timeout-method thread -k "h2p_gemm_gather" > $O/nn4_tests.log 2>&1 || { echo "nn4 tests failed"; tail -30 $O/nn4_tests.log; exit 1; }
tail -2 $O/nn4_tests.log
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
NTS_AGG_LDS=0 timeout -k 10 300 python -u bench.py $B > $O/bench_reg.json 2> $O/bench_reg.err || { echo "bench reg failed"; tail -5 $O/bench_reg.err; exit 1; }
timeout -k 10 300 python -u bench.py $B > $O/bench_lds.json 2> $O/bench_lds.err || { echo "bench lds failed"; tail -5 $O/bench_lds.err; exit 1; }
NTS_H2_NN4=1 timeout -k 10 300 python -u bench.py $B > $O/bench_nn4.json 2> $O/bench_nn4.err || { echo "bench nn4 failed"; tail -5 $O/bench_nn4.err; exit 1; }
NTS_GEMM_CUS=232 timeout -k 10 300 python -u bench.py $B > $O/bench_cus232.json 2> $O/bench_cus232.err || { echo "bench cus failed"; tail -5 $O/bench_cus232.err; exit 1; }
python - <<PY
import json
for f in ("$O/bench.json", "$O/bench_reg.json", "$O/bench_lds.json", "$O/bench_nn4.json", "$O/bench_cus232.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 4), "ms/step", {k: (round(v["avg_launch_ms"]*1e3,1), round(v["frac"],3)) for k, v in d["roofline"].get("kernels", {}).items()}, d["config"].get("training_stream_alone"))
PY
bash scripts/pmc_stalls.sh $T > $O/stalls.txt 2>&1 || { tail -5 $O/stalls.txt; exit 1; }
cat $O/stalls.txt
