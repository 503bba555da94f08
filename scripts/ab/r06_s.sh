#!/bin/bash
# the sampler / full-size / host suites in one process, product build vs
# lib_csr2, alternating (an intermittent host-test mismatch: which build?)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06w; mkdir -p $O
export TMPDIR=/tmp
for v in base csr2 base; do
  if [ $v = base ]; then L=; else L=scripts/probe/lib_$v/libnts_hip.so; fi
  NTS_HIP_LIB=$L timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
      tests/test_hip_kernels.py tests/test_fullsize.py tests/test_host.py >> $O/tests_$v.log 2>&1
  echo "$v rc=$?" >> $O/rc.txt
done
