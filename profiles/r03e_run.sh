#!/bin/bash
# r03e: interleaved A/B of the peer count from which device-resident module rounds take the table
# path (ACCDFL_AMD_MULTI_TABLE_MIN_PEERS=1: every round; 33: rounds of > 32 peers), after the reduce
# was moved ahead of the module clone in _device_round.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03e
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "multi_table or device_modules or multi_tensor or fedavg_device or tied or center_copy" > $out/tests.log 2>&1 &&
for r in 1 2; do
  for mp in 1 33; do
    ACCDFL_AMD_MULTI_TABLE_MIN_PEERS=$mp timeout -k 10 300 python -u bench.py --device-configs-only \
      > $out/dev_mp${mp}_r${r}.log 2>&1 || exit 1
  done
done
