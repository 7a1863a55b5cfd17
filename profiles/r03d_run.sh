#!/bin/bash
# r03d: dla_wsum_multi_table with the two-level workgroup -> tensor search; parity, then an
# interleaved A/B of the search (DLA_MULTI_SEARCH=1 two-level count, 0 binary search) on the
# device-resident module rounds.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03d
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "multi_table or device_modules or multi_tensor or fedavg_device" > $out/tests.log 2>&1 &&
for r in 1 2; do
  for se in 1 0; do
    DLA_MULTI_SEARCH=$se timeout -k 10 300 python -u bench.py --device-configs-only > $out/dev_s${se}_r${r}.log 2>&1 || exit 1
  done
done
