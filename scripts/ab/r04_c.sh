#!/bin/bash
# Round-4 batch C: tests, sampler traces (C2, C3), C2 bench, MT traces
# (default walker choice and every layer chunked), streaming probe, C3/C4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04c2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c2 or c3 or c4" > $O/full.log 2>&1 || { echo "fullsize tests failed"; tail -30 $O/full.log; exit 1; }
tail -1 $O/full.log
bash scripts/prof_sampler.sh $(basename $O)_samp > $O/samp.txt 2>&1 || { tail -5 $O/samp.txt; exit 1; }
head -14 $O/samp.txt
bash scripts/prof_sampler.sh $(basename $O)_samp3 --shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean > $O/samp3.txt 2>&1 || { tail -5 $O/samp3.txt; exit 1; }
head -16 $O/samp3.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 8 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
a = d["config"].get("training_stream_alone") or {}
print("C2", round(d["ms_per_step"], 4), "ms/step; alone", round(a.get("ms_per_step", 0), 4), a.get("kernel_avg_us"), "sampler-only %.3g" % d["config"]["gpu_sampler_only"]["value"])
PY
for m in def ch; do
  if [ $m = ch ]; then E="NTS_MT_CHUNKED=1"; else E="NTS_NONE=0"; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mt_$m -o run --output-format csv -- python3 bench.py --rng mt --steps 6 --warmup 2 --no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0 --no-interference-probe > $O/mt_$m.json 2> $O/mt_$m.err || { echo "mt $m failed"; tail -5 $O/mt_$m.err; exit 1; }
  python3 - $O $m <<'PY'
import csv, glob, json, sys
o, m = sys.argv[1], sys.argv[2]
d = json.loads(open(f"{o}/mt_{m}.json").read().strip().splitlines()[-1])
print("MT", m, round(d["ms_per_step"], 3), "ms/step")
f = glob.glob(f"{o}/mt_{m}/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:9]:
    print("  %-60s calls=%-4s avg_us=%.1f pct=%s" % (r["Name"].split("(")[0][-60:], r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"]))
PY
done
timeout -k 10 120 scripts/probe/stream_probe 10 > $O/stream.txt 2>&1 || { echo "probe failed"; tail -5 $O/stream.txt; exit 1; }
cat $O/stream.txt
for v in product nn3acc2 product nn3acc2; do
  if [ $v = product ]; then L="NTS_NONE=0"; else L="NTS_HIP_LIB=scripts/probe/lib_$v/libnts_hip.so"; fi
  env $L timeout -k 10 200 python -u scripts/micro_bottom.py > $O/mb_$v.json 2> $O/mb_$v.err || { echo "micro_bottom $v failed"; tail -5 $O/mb_$v.err; exit 1; }
  echo "$v $(cat $O/mb_$v.json)"
done
NTS_HIP_LIB=scripts/probe/lib_nn3acc2/libnts_hip.so timeout -k 10 300 python -u -m pytest tests/test_gemm_h2.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/acc2_tests.log 2>&1 || { echo "acc2 tests failed"; tail -20 $O/acc2_tests.log; exit 1; }
tail -1 $O/acc2_tests.log
bash scripts/bench_configs.sh r04c || exit 1
