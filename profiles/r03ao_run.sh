#!/bin/bash
# r03ao: the many-tensor kernel with 4 blocks of 64 vectors per workgroup for rounds of >= 256 MiB
# (DLA_MULTI_BV): the multi-tensor / device-module GPU tests with BV forced to 4 (every size) and at
# the default, the whole suite, then the device-resident module rounds at BV 1 / 4, interleaved twice.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ao
mkdir -p $out
DLA_MULTI_BV=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "multi or device or layouts or call_sites or tied or fedavg" > $out/tests_bv4.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit $?
for r in 1 2; do
  for bv in 1 4; do
    DLA_MULTI_BV=$bv timeout -k 10 300 python -u bench.py --device-configs-only > $out/dev_bv${bv}_r${r}.log 2>&1 || exit $?
  done
done
