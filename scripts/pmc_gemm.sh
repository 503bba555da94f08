#!/bin/bash
# PMC passes over scripts/one_gemm.py (each counter group in its own run)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm${PMC_TAG:-}
mkdir -p $OUT
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_CYCLES" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 scripts/one_gemm.py "$@" > $OUT/p$i.log 2>&1
done
echo done
