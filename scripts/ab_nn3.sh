#!/bin/bash
# The planar pair-table GEMMs alone (scripts/micro_bottom.py; NTS_NN3_DIAG=4 =
# the runtime-step-count NN loop), their tests, then scripts/gpu_check.sh.
O=gpurun_out/${1:-abnn}
mkdir -p $O
for e in "NTS_NN3_DIAG=4" "" "NTS_NN3_DIAG=4" ""; do
  env $e timeout -k 10 120 python3 scripts/micro_bottom.py --iters 30 >> $O/ab.jsonl 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gemm_h2.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
bash scripts/gpu_check.sh ${1:-abnn}_chk
