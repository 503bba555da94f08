#!/bin/bash
# A/B of knobs on the headline bench (no CPU baseline).  usage: overlap_ab.sh "ENV|flags" ...
set -o pipefail
mkdir -p gpurun_out
for spec in "$@"; do
  e=${spec%%|*}; f=${spec#*|}
  env X=1 $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $f > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo FAILED "$spec"; tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));c=d['config'];print('$spec', round(d['ms_per_step'],3),'ms', round(d['value']/1e6),'M/s agg', round(d['roofline']['avg_launch_ms'],3), 'sampler', round(1e3*c.get('sampler_s_per_step',0),3), 'issue', round(1e3*c.get('host_train_issue_s_per_step',0),3))"
done
