#!/bin/bash
# the driver's round-end smoke entry on the final library
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05aq
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05aq/smoke.log 2>&1
