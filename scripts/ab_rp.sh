#!/bin/bash
# A/B of a pair-table GEMM knob (default: the row-aligned LDS-DMA pieces,
# NTS_NN3_RP=0 NTS_TN4_RP=0) alone (micro_bottom) and in the C2 bench; their tests first.
#   scripts/ab_rp.sh <tag> "<ENV=VAL ...>"
O=gpurun_out/${1:-rp}
AB=${2:-NTS_NN3_RP=0 NTS_TN4_RP=0}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_h2.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for e in "$AB" "" "$AB" ""; do
  env $e timeout -k 10 120 python3 scripts/micro_bottom.py --iters 30 >> $O/ab.jsonl 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
done
cat $O/ab.jsonl
i=0
for e in "$AB" "" "$AB" ""; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --epochs 1 --steps 40 > $O/c2_$i.json 2> $O/c2_$i.err || { echo "bench failed ($e)"; tail -20 $O/c2_$i.err; exit 1; }
  python3 - $O/c2_$i.json "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(repr(sys.argv[2]), round(d["ms_per_step"], 4), {k: round(v["avg_launch_ms"] * 1e3, 1) for k, v in d["roofline"]["kernels"].items()})
PY
done
