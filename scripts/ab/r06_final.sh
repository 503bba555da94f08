#!/bin/bash
# round-6 record: full GPU suite, the default bench line, then the trace and
# PMC passes (profiles/collect.sh) on the same library
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.log || exit 1
bash profiles/collect.sh r06 20 && bash scripts/bench_configs.sh r06final > $O/configs.txt 2>&1 && bash scripts/bench_c5.sh r06 > $O/c5.txt 2>&1
