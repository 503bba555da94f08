#!/bin/bash
# v1 split-GEMM timing probes (NTS_S3_DIAG bits; results numerically invalid)
set -o pipefail
O=gpurun_out/diag_v1_${1:-a}
mkdir -p $O
for d in 0 1 2 4 8 16 3 24; do
  NTS_S3_V1=1 NTS_S3_DIAG=$d timeout -k 10 120 python -u scripts/micro_split3.py > $O/d$d.log 2>&1 || { echo "diag $d failed"; tail -5 $O/d$d.log; exit 1; }
  echo "diag $d: $(grep split3 $O/d$d.log)"
done
