#!/bin/bash
# rocprofv3 kernel trace of scripts/micro_h2.py (per-kernel times of the GEMM paths)
export TMPDIR=/tmp
O=gpurun_out/${1:-h2g}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python3 scripts/micro_h2.py --iters 5 > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:100], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
