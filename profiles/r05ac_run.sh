#!/bin/bash
# Round 5: the seeded fuzz of FedAvg.aggregate against the C oracle (tests/test_fuzz_fedavg.py), then
# the whole GPU suite on the fixed tree.
set -o pipefail
mkdir -p gpurun_out/r05ac
timeout -k 10 600 python -u -m pytest tests/test_fuzz_fedavg.py -m gpu -q --timeout 120 --timeout-method thread -rf \
  > gpurun_out/r05ac/fuzz.log 2>&1 || { tail -30 gpurun_out/r05ac/fuzz.log; exit 1; }
tail -3 gpurun_out/r05ac/fuzz.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05ac/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r05ac/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r05ac/gpu_tests.log
