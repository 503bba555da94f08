#!/bin/bash
# C2 headline bench with and without an env knob, alternating, plus one
# kernel trace of each (rocprofv3 --kernel-trace --stats): the knob's kernel time.
#   scripts/ab_c2.sh <tag> "<ENV=VAL ...>" [kernel-name-regex]
O=gpurun_out/${1:-abc2}
E=${2:-NTS_DUMMY=1}
R=${3:-top_xent}
mkdir -p $O
export TMPDIR=/tmp
i=0
for e in "" "$E" "" "$E"; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --epochs 1 > $O/c2_$i.json 2> $O/c2_$i.err || { echo "c2 failed ($e)"; tail -20 $O/c2_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/c2_$i.json').read().strip().splitlines()[-1]); print(repr('$e'), round(d['ms_per_step'], 4))"
done
for e in "" "$E"; do
  i=$((i+1))
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary-af --epochs 0 --steps 20 --warmup 3 > $O/p_$i.json 2> $O/p_$i.err || { echo "trace failed ($e)"; tail -20 $O/p_$i.err; exit 1; }
  f=$(ls $O/tr_$i/*/run_kernel_stats.csv $O/tr_$i/run_kernel_stats.csv 2>/dev/null | head -1)
  echo "trace $i ($e):"; grep -E "$R" "$f" | cut -c1-150
done
