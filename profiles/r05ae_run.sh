#!/bin/bash
# Round 5: the DeviceModelManager fuzz (tests/test_fuzz_model_manager.py) on the GPU.
set -o pipefail
mkdir -p gpurun_out/r05ae
timeout -k 10 600 python -u -m pytest tests/test_fuzz_model_manager.py -m gpu -q --timeout 120 --timeout-method thread -rf \
  > gpurun_out/r05ae/fuzz_mm.log 2>&1; rc=$?
tail -60 gpurun_out/r05ae/fuzz_mm.log; exit $rc
