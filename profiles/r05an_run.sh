#!/bin/bash
# Round 5: random-shape sharding cases with the HIP reducer (gloo ranks sharing the GPU).
set -o pipefail
mkdir -p gpurun_out/r05an
timeout -k 10 600 python -u -m pytest tests/test_sharding_gloo.py -m gpu -k random -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05an/sharding.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/r05an/sharding.log | cut -c1-250 | tail -20; exit $rc
