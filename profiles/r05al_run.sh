#!/bin/bash
# Round 5: the fuzzers with tied parameters (FedAvg.aggregate and DeviceModelManager) on the GPU.
set -o pipefail
mkdir -p gpurun_out/r05al
timeout -k 10 600 python -u -m pytest tests/test_fuzz_fedavg.py tests/test_fuzz_model_manager.py -m gpu -q \
  --timeout 200 --timeout-method thread -rf > gpurun_out/r05al/fuzz.log 2>&1; rc=$?
grep -E "^E +AssertionError|^E +[A-Za-z]+Error|passed|failed" gpurun_out/r05al/fuzz.log | cut -c1-300 | tail -30; exit $rc
