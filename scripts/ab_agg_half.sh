#!/bin/bash
# A/B of the 16-lane x 2-vector shape for 128-float rows (NTS_AGG_HALF=1):
# aggregation tests with the knob, then C2 (bench + traces) and C3/C4.
O=gpurun_out/${1:-agghalf}
mkdir -p $O
NTS_AGG_HALF=1 timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_fullsize.py tests/test_host.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
bash scripts/ab_c2.sh ${1:-agghalf}_c2 "NTS_AGG_HALF=1" "k_spmm_gather" || exit 1
bash scripts/ab_c3.sh ${1:-agghalf}_c3 "NTS_AGG_HALF=1"
