#!/bin/bash
# Counter passes over scripts/prof_gemm.py (one rocprofv3 run per counter set).
set -e
export TMPDIR=/tmp
O=gpurun_out/pmc_gemm
mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 scripts/prof_gemm.py > $O/t.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES -d $O/p1 -o run --output-format csv -- python3 scripts/prof_gemm.py > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA -d $O/p2 -o run --output-format csv -- python3 scripts/prof_gemm.py > $O/p2.log 2>&1 || echo p2 failed
echo done
