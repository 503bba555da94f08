#!/bin/bash
# GPU suite, then C3/C4 with NTS_H2D=0 A/B (scripts/ab_c3.sh)
O=gpurun_out/${1:-s3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/ab_c3.sh ${1:-s3}_c3 NTS_H2D=0
