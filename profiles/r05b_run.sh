#!/bin/bash
# r05b: new round-5 tests on the GPU: mixed-dtype parity (dla_wsum_mixed, ABI v13) and the bf16 /
# 8-rank gloo sharding rehearsal with the HIP reducer.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05b
mkdir -p $out
run() {
  local t=$1; shift
  echo "$(date +%T) start: $*" >> $out/steps.log
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$(date +%T) rc=$rc: $*" >> $out/steps.log
  case $rc in 124|137|134|139) exit $rc;; esac
  return 0
}
run 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "mixed" --timeout 120 --timeout-method thread > $out/mixed_tests.log 2>&1
run 600 python -u -m pytest tests/test_sharding_gloo.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/sharding_tests.log 2>&1
