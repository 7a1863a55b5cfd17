#!/bin/bash
# Round 5: the GPU suite and smoke on the final tree (after the tied-parameter fuzz).
set -o pipefail
mkdir -p gpurun_out/r05am
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05am/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r05am/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r05am/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05am/smoke.log 2>&1; rc=$?
tail -1 gpurun_out/r05am/smoke.log; exit $rc
