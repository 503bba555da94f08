#!/bin/bash
# Narrow-layer weight gradient (k_gemm_tn_big, 128-row tile): blocks per launch
# A/B alone (micro_layer f32_tn_masked_us) and in C3 / C4.
#   scripts/ab_narrow.sh <tag> "<values>" "<C3 A/B env>"
O=gpurun_out/${1:-narrow}
V=${2:-256 512 768 1024}
mkdir -p $O
NTS_TN_NARROW_BLOCKS=512 timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -k gemm -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  for v in $V; do
    NTS_TN_NARROW_BLOCKS=$v timeout -k 10 120 python3 scripts/micro_layer.py --iters 30 > $O/m_$v.json 2>> $O/m.err || { tail -20 $O/m.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/m_$v.json')); print($v, d['f32_tn_masked_us'], d['split3_tn_masked_us'])"
  done
done
E=${3:-}
[ -z "$E" ] && exit 0
bash scripts/ab_c3.sh ${1:-narrow}_c3 "$E"
