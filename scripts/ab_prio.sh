#!/bin/bash
# C2 bench: the sampler stream at high priority (default) vs normal (--no-priority)
O=gpurun_out/${1:-prio}
mkdir -p $O
i=0
for a in "" "--no-priority" "" "--no-priority" "" "--no-priority"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --epochs 0 --sampler-batches 0 --steps 60 $a > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
  python3 - $O/b$i.json "$a" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(repr(sys.argv[2]), round(d["ms_per_step"], 4))
PY
done
