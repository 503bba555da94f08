#!/bin/bash
# Timing probes of the planar pair-table GEMMs alone (scripts/micro_bottom.py):
# full kernels, then without MFMAs / without streaming / without slab stores.
O=gpurun_out/${1:-diagb}
mkdir -p $O
for e in "" "NTS_NN3_DIAG=1 NTS_TN4_DIAG=1" "NTS_NN3_DIAG=2 NTS_TN4_DIAG=2" "NTS_TN4_DIAG=4"; do
  env $e timeout -k 10 120 python3 scripts/micro_bottom.py --iters 20 >> $O/diag.jsonl 2>> $O/diag.err || { tail -20 $O/diag.err; exit 1; }
done
cat $O/diag.jsonl
