set -o pipefail
mkdir -p gpurun_out/r04fs
timeout -k 10 400 python -u -m pytest tests/test_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread --durations=10 > gpurun_out/r04fs/full.log 2>&1 || { echo "fullsize failed"; grep -v "^  File\|^    " gpurun_out/r04fs/full.log | tail -30; exit 1; }
grep -E "passed|failed|s call" gpurun_out/r04fs/full.log
