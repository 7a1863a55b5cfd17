#!/bin/bash
# r03b: the whole GPU suite (the vec kernels now take their peer pointers as global-address-space
# pointers; dla_wsum_multi_table is new), then the device-resident module rounds.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03b
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --device-configs-only > $out/device_configs.log 2>&1
