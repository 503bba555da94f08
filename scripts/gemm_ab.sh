#!/bin/bash
# A/B of GEMM kernel variants (env specs) on the GPU box
set -o pipefail
for spec in "$@"; do
  env X=1 $spec timeout -k 10 120 python scripts/micro_gemm3.py || { echo FAILED "$spec"; exit 1; }
done
