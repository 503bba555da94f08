#!/bin/bash
# engine counters of the fp32-exact bottom-layer GEMMs (micro_x3.py, C2 size)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05e; mkdir -p $O
export TMPDIR=/tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $O/p1 -o run -- \
    python3 scripts/micro_x3.py --iters 10 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d $O/p2 -o run -- \
    python3 scripts/micro_x3.py --iters 10 > $O/p2.log 2>&1 || exit 1
