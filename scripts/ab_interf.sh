#!/bin/bash
# How much the pipelined sampler costs the C2 step: the bench as is, with the
# training stream alone (NTS_DIAG_REUSE_SAMPLE=1, diagnostic), and with the
# sampler stream masked to a CU subset.
O=gpurun_out/${1:-interf}
mkdir -p $O
i=0
for a in "" "DIAG" "--sampler-cus 32" "" "DIAG" "--sampler-cus 64"; do
  i=$((i+1))
  if [ "$a" = "DIAG" ]; then
    NTS_DIAG_REUSE_SAMPLE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --epochs 0 --sampler-batches 0 --steps 40 > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
  else
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary-af --epochs 0 --sampler-batches 0 --steps 40 $a > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
  fi
  python3 - $O/b$i.json "$a" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print(repr(sys.argv[2]), round(d["ms_per_step"], 4), "host wait", round(c.get("host_sampler_wait_s_per_step", 0) * 1e3, 3), "issue", round(c.get("host_train_issue_s_per_step", 0) * 1e3, 3))
PY
done
