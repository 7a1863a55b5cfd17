#!/bin/bash
# r06fz: the 16x fuzz campaign (FedAvg.aggregate, C ABI, DeviceModelManager against the C oracle) on the
# final tree, after the walk / tree-clone changes.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06fz
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
export ACCDFL_AMD_FUZZ_SCALE=16
run 1100 python -u -m pytest tests/test_fuzz_fedavg.py tests/test_fuzz_abi.py tests/test_fuzz_model_manager.py -m gpu -q --timeout 300 --timeout-method thread -rs > $out/fuzz.log 2>&1
