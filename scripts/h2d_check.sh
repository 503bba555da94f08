#!/bin/bash
# k_h2_nnd: its tests, the layer micro benchmark, then C3/C4 with NTS_H2D=0 A/B.
O=gpurun_out/${1:-h2d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_h2.py -x -q --timeout 120 --timeout-method thread -k "h2d" > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python3 scripts/micro_layer.py > $O/micro.json 2> $O/micro.err || { tail -20 $O/micro.err; exit 1; }
cat $O/micro.json
bash scripts/ab_c3.sh ${1:-h2d}_c3 NTS_H2D=0
