#!/bin/bash
# The default bench line with the reference-stream secondary.
set -o pipefail
O=gpurun_out/${1:-r04q}
mkdir -p $O
start=$(date +%s)
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
echo "bench took $(( $(date +%s) - start )) s"
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['config']['reference_stream_secondary'])"
