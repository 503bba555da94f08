#!/bin/bash
# Round-4 measurement batch: kernel tests, the aggregation micro benchmark on
# the product build and the compile-time A/B builds (scripts/probe/lib_*:
# `make -C sample-based-gnn_amd/csrc variant V=... VFLAGS=...`), the streaming
# probe of the pair table (scripts/probe/stream_probe), the pair-table GEMMs
# alone, the sampler trace, a C2 bench and the C3/C4 config benches.
set -o pipefail
O=gpurun_out/${1:-r04probe}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in product pf0 pf1 pf2w6; do
  if [ $v = product ]; then L=""; else L="NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so"; fi
  env $L timeout -k 10 200 python -u scripts/micro_agg.py > $O/micro_agg_$v.json 2> $O/micro_agg_$v.err || { echo "micro_agg $v failed"; tail -5 $O/micro_agg_$v.err; exit 1; }
  echo "$v $(cat $O/micro_agg_$v.json)"
done
timeout -k 10 120 scripts/probe/stream_probe 10 > $O/stream.txt 2>&1 || { echo "probe failed"; tail -5 $O/stream.txt; exit 1; }
cat $O/stream.txt
timeout -k 10 200 python -u scripts/micro_bottom.py > $O/micro_bottom.json 2> $O/micro_bottom.err || { echo "micro_bottom failed"; tail -5 $O/micro_bottom.err; exit 1; }
cat $O/micro_bottom.json
bash scripts/prof_sampler.sh $(basename $O)_samp > $O/samp.txt 2>&1 || { tail -5 $O/samp.txt; exit 1; }
head -14 $O/samp.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 8 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = d["config"].get("training_stream_alone") or {}
print("C2", round(d["ms_per_step"], 4), "ms/step; alone", round(a.get("ms_per_step", 0), 4), a.get("kernel_avg_us"), "sampler-only %.3g" % d["config"]["gpu_sampler_only"]["value"])
PY
bash scripts/bench_configs.sh r04 || exit 1
