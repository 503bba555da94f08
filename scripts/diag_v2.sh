#!/bin/bash
# NN v2 timing probes (compile-time variants; results numerically invalid):
# 1 no global loads, 2 no split, 4 no LDS B reads, 8 no barrier, 3, 15 MFMA only
set -o pipefail
for d in 0 1 2 4 8 3 15; do
  NTS_S3_NN2=1 NTS_S3_DIAG=$d timeout -k 10 60 python -u scripts/diag_split3.py 2>&1 | grep diag || exit 1
done
NTS_S3_V1=1 timeout -k 10 60 python -u scripts/diag_split3.py 2>&1 | grep diag
