#!/bin/bash
# PMC passes over scripts/prof_split3.py (one rocprofv3 run per counter group).
set -e
export TMPDIR=/tmp
O=gpurun_out/pmc_s3_${1:-a}
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 scripts/prof_split3.py > $O/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL --kernel-trace -d $O/p1 -o run --output-format csv -- python3 scripts/prof_split3.py > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --kernel-trace -d $O/p2 -o run --output-format csv -- python3 scripts/prof_split3.py > $O/p2.log 2>&1
echo done
