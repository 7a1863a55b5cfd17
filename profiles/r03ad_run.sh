#!/bin/bash
# r03ad: the occupancy cap extended to 9-15 peers (tiled) and to the kernels over separate peer
# buffers (row-major vector kernel, many-tensor table kernel): the GPU suite, then the device-resident
# module rounds with the separate-buffer cap on (policy) and off (DLA_VEC_CAP_ROWS=0), interleaved twice.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ad
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit $?
for r in 1 2; do
  for c in 1 0; do
    DLA_VEC_CAP_ROWS=$c timeout -k 10 300 python -u bench.py --device-configs-only > $out/dev_cap${c}_r${r}.log 2>&1 || exit $?
  done
done
