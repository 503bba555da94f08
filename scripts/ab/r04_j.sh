#!/bin/bash
# Round-4 batch J: k_h2_nn3 in 1, 2 or 3 rounds of blocks over the CUs
# (NTS_NN3_WAVES) — the pipelined sampler's blocks hold CUs the one-block-per-CU
# forward GEMM then waits on.  NN tests at 2, then C2 benches, twice each.
set -o pipefail
O=gpurun_out/${1:-r04j}
mkdir -p $O
NTS_NN3_WAVES=2 timeout -k 10 300 python -u -m pytest tests/test_gemm_h2.py tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
for w in 1 2 3 1 2 3; do
  NTS_NN3_WAVES=$w timeout -k 10 300 python -u bench.py $B > $O/b_$w.json 2> $O/b_$w.err || { echo "bench $w failed"; tail -5 $O/b_$w.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$w.json').read().strip().splitlines()[-1]); a=d['config'].get('training_stream_alone') or {}; k=d['roofline']['kernels']; print('waves $w C2', round(d['ms_per_step'],4), 'alone', round(a.get('ms_per_step',0),4), {n: round(v['avg_launch_ms']*1e3,1) for n, v in k.items()}, a.get('kernel_avg_us'))"
done
