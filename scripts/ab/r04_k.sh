#!/bin/bash
# Round-4 batch K: k_h2_tn4's X stage swizzled by 4 (row & 3) (conflict-free
# A^T reads): the pair-table GEMM and host tests, C2 benches, and the LDS
# bank-conflict counter of the bench's kernels.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04k}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_h2.py tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="--no-cpu-baseline --no-secondary-af --no-secondary-exact --epochs 0 --sampler-batches 0"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py $B > $O/b_$i.json 2> $O/b_$i.err || { echo "bench $i failed"; tail -5 $O/b_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b_$i.json').read().strip().splitlines()[-1]); a=d['config'].get('training_stream_alone') or {}; print('C2', round(d['ms_per_step'],4), 'alone', round(a.get('ms_per_step',0),4), a.get('kernel_avg_us'))"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace -d $O/sq -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 $B > $O/sq.log 2>&1 || { echo "pmc failed"; tail -5 $O/sq.log; exit 1; }
python3 - $O/sq <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for row in csv.DictReader(open(f[0])):
    k = row.get("Kernel_Name", "")
    if "h2_tn4" in k or "h2_nn3" in k:
        agg[k[:40]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: sorted(v)[len(v) // 2] for c, v in d.items()})
PY
