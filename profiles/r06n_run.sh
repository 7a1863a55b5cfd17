#!/bin/bash
# r06n: the device round's parameters made in two halves (walk.cpp param_blocks before the launch, param_wrap
# while the reduce runs): the device-round GPU tests, smoke, and the host/GPU split with the one-step A/B.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06n
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
run 600 python -u -m pytest tests/test_gpu_parity.py tests/test_center_copy_layouts.py tests/test_call_sites.py tests/test_fuzz_fedavg.py -m gpu -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 120 python -u profiles/r06_device_round_split.py > $out/device_round_split.jsonl 2>&1
run 120 python -u profiles/r06_device_round_split.py >> $out/device_round_split.jsonl 2>&1
run 120 python -u profiles/r06_result_alloc_probe.py > $out/result_alloc.jsonl 2>&1
