#!/bin/bash
# Round-4 interference A/B: the single-pass frontier compaction's tests, then
# C2 benches with the stream priorities swapped (--training-priority: the
# training stream high, the sampler's normal), both normal (--no-priority),
# and a CU split (--sampler-cus n with the pair-table GEMM grids narrowed to
# the training stream's 256 - n CUs, NTS_GEMM_CUS), each twice.
set -o pipefail
T=${1:-r04prio}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_presample_golden.py tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2 or c3 or c4" > $O/full.log 2>&1 || { echo "fullsize tests failed"; tail -30 $O/full.log; exit 1; }
tail -1 $O/full.log
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
run() {  # tag env args...
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python -u bench.py $B "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo "bench $tag failed"; tail -5 $O/bench_$tag.err; exit 1; }
  python3 - $O/bench_$tag.json "$tag" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = d["config"].get("training_stream_alone") or {}
print(sys.argv[2], round(d["ms_per_step"], 4), "ms/step; alone", round(a.get("ms_per_step", 0), 4),
      {k: v for k, v in (a.get("kernel_avg_us") or {}).items()})
PY
}
run def1 NTS_NONE=0
run tprio1 NTS_NONE=0 --training-priority
run noprio1 NTS_NONE=0 --no-priority
run cus32_1 NTS_GEMM_CUS=224 --sampler-cus 32
run cus16_1 NTS_GEMM_CUS=240 --sampler-cus 16
run def2 NTS_NONE=0
run tprio2 NTS_NONE=0 --training-priority
# the reference-stream sampler: the default walker choice, and the seed layer chunked too
run mt NTS_NONE=0 --rng mt --steps 10 --warmup 2 --no-interference-probe
run mtch NTS_MT_CHUNKED=1 --rng mt --steps 10 --warmup 2 --no-interference-probe
bash scripts/prof_sampler.sh ${T}_samp > $O/samp.txt 2>&1 || { tail -5 $O/samp.txt; exit 1; }
head -16 $O/samp.txt
echo done
