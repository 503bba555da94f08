#!/bin/bash
# test_host's transform-first vs aggregate-first step with dropout: the product
# build (bucket CSR transpose) and lib_csr2 (two-pass radix + finalize), 3x each
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06v; mkdir -p $O
export TMPDIR=/tmp
for v in base csr2 base csr2; do
  if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
  NTS_HIP_LIB=$L timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
      tests/test_host.py -k "transform_first_trains or unfused or gat" >> $O/tests_$v.log 2>&1
  echo "$v rc=$?" >> $O/rc.txt
done
