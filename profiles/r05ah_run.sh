#!/bin/bash
# Round 5: the dla_mean fuzz and the concurrent device-round test on the GPU.
set -o pipefail
mkdir -p gpurun_out/r05ah
timeout -k 10 600 python -u -m pytest tests/test_fuzz_abi.py tests/test_fuzz_fedavg.py -m gpu -k "mean or concurrent" -q \
  --timeout 200 --timeout-method thread -rf > gpurun_out/r05ah/fuzz.log 2>&1; rc=$?
tail -40 gpurun_out/r05ah/fuzz.log; exit $rc
