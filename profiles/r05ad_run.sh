#!/bin/bash
# Round 5: the C-ABI fuzz (tests/test_fuzz_abi.py) on the GPU.
set -o pipefail
mkdir -p gpurun_out/r05ad
timeout -k 10 600 python -u -m pytest tests/test_fuzz_abi.py -m gpu -q --timeout 120 --timeout-method thread -rf \
  > gpurun_out/r05ad/fuzz_abi.log 2>&1; rc=$?
tail -30 gpurun_out/r05ad/fuzz_abi.log; exit $rc
