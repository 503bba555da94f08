#!/bin/bash
# Round-4 end evidence, part A (committed build): the whole GPU suite, smoke,
# the default bench line and the reference-order (aggregate-first) line.
set -o pipefail
bash scripts/gpu_check.sh ${1:-r04} || exit 1
