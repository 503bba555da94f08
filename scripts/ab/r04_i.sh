#!/bin/bash
# Round-4 batch I: the post-mask gather's rows in flight (scripts/probe/lib_pmu2,
# lib_pmu4) against the product build — micro benchmark, C2 bench (TESTS="pmu2 pmu4"
# runs the kernel tests on them first; pmu2 is not bit-equal to the plain
# backward gather in test_spmm_csr_bwd_postmask[41]).
set -o pipefail
O=gpurun_out/${1:-r04i}
mkdir -p $O
for v in ${TESTS:-}; do
  NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -20 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
done
for v in product pmu2 pmu4 product pmu2 pmu4; do
  if [ $v = product ]; then L="NTS_NONE=0"; else L="NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so"; fi
  env $L timeout -k 10 200 python -u scripts/micro_agg.py > $O/ma_$v.json 2> $O/ma_$v.err || { echo "micro_agg $v failed"; tail -5 $O/ma_$v.err; exit 1; }
  python3 -c "import json; a=json.load(open('$O/ma_$v.json')); print('$v', 'bottom', a['bottom']['fwd_us'], a['bottom']['bwd_us'], 'hop0', a['hop0']['fwd_us'], a['hop0']['bwd_us'])"
done
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
for v in product pmu2 pmu4 product pmu2 pmu4; do
  if [ $v = product ]; then L="NTS_NONE=0"; else L="NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so"; fi
  env $L timeout -k 10 300 python -u bench.py $B > $O/b_$v.json 2> $O/b_$v.err || { echo "bench $v failed"; tail -5 $O/b_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); a=d['config'].get('training_stream_alone') or {}; print('$v C2', round(d['ms_per_step'],4), 'alone', round(a.get('ms_per_step',0),4))"
done
