#!/bin/bash
# (1) row-access-order probe of the NN's A stream (scripts/probe/rowpat_probe.hip);
# (2) k_x3_tn timing probes (probe build, NTS_X3_DIAG: 1 no MFMA, 2 no splits,
#     4 no DMA after the prologue, 8 no A fragment reads, 32 no slab stores)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 ./scripts/probe/rowpat_probe > $O/rowpat.jsonl || exit 1
for r in 1 2; do
  for d in 0 1 2 4 8 32 6 10 14; do
    NTS_HIP_LIB=scripts/probe/lib/libnts_hip.so NTS_X3_DIAG=$d timeout -k 10 120 python -u scripts/micro_x3.py --iters 30 --tag diag$d >> $O/micro.jsonl 2>> $O/micro.log || exit 1
  done
done
