#!/bin/bash
# k_x3_nn7 timing probes (probe build, NTS_X3_DIAG: 1 no MFMA, 2 no split, 4 no
# A loads, 8 no B reads, 16 no W DMA, 32 no barrier) and the B fragments two
# column tiles ahead (lib_bq2) vs one (product)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for d in 0 1 2 4 8 16 32 6 14 62 63; do
    NTS_HIP_LIB=scripts/probe/lib/libnts_hip.so NTS_X3_DIAG=$d timeout -k 10 120 python -u scripts/micro_x3.py --iters 30 --tag diag$d >> $O/micro.jsonl 2>> $O/micro.log || exit 1
  done
  for v in base bq2; do
    if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
    NTS_HIP_LIB=$L timeout -k 10 120 python -u scripts/micro_x3.py --iters 30 --tag $v >> $O/micro.jsonl 2>> $O/micro.log || exit 1
  done
done
