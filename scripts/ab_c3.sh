#!/bin/bash
# C3 (products-shaped GraphSAGE 100-256-256-47, 15-10-5, B=1024) and C4
# (100-256-47, 25-10) bench lines with and without an env knob:
#   scripts/ab_c3.sh <tag> "<ENV=VAL ...>"
O=gpurun_out/${1:-abc3}
E=${2:-NTS_H2_DYN=1}
mkdir -p $O
C3="--shape products --layers 100-256-256-47 --fanout 15-10-5 --batch 1024 --weight mean"
C4="--shape products --layers 100-256-47 --fanout 25-10 --batch 1024"
i=0
for e in "" "$E" "" "$E"; do
  i=$((i+1))
  env $e timeout -k 10 300 python -u bench.py $C3 --steps 40 --warmup 10 --no-cpu-baseline --no-secondary-af --epochs 0 --sampler-batches 0 > $O/c3_$i.json 2> $O/c3_$i.err || { echo "c3 failed ($e)"; tail -20 $O/c3_$i.err; exit 1; }
  env $e timeout -k 10 300 python -u bench.py $C4 --steps 40 --warmup 10 --no-cpu-baseline --no-secondary-af --epochs 0 --sampler-batches 0 > $O/c4_$i.json 2> $O/c4_$i.err || { echo "c4 failed ($e)"; tail -20 $O/c4_$i.err; exit 1; }
  python3 - "$O" $i "$e" <<'PY'
import json, sys
o, i, e = sys.argv[1], sys.argv[2], sys.argv[3]
for c in ("c3", "c4"):
    d = json.loads(open(f"{o}/{c}_{i}.json").read().strip().splitlines()[-1])
    print(c, repr(e), round(d["ms_per_step"], 4), "ms/step", "%.4g" % d["value"])
PY
done
