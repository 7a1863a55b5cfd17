#!/bin/bash
# r06b: native wire ingress (csrc/walk.cpp scan_state_dict + one batched gather + one slab copy per peer):
# the wire / DFL / manager-fuzz GPU tests, then the default bench (dfl_round_layout ingress_GBps, its
# reference-style leg and phase split).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06b
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
run 600 python -u -m pytest tests/test_wire.py tests/test_gpu_dfl_round.py tests/test_fuzz_model_manager.py tests/test_call_sites.py -m gpu -x -q --timeout 300 --timeout-method thread -rs > $out/gpu_tests.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
