#!/bin/bash
# r06d: staged-on-arrival rows with the native parameter fingerprint, the call-site
# tests through DeviceModelManager, allocator-visible device results (the whole GPU suite), and the
# granularity probe with the staggered-contiguous variant.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06d
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
run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > $out/gpu_tests.log 2>&1
run 300 python -u profiles/r06_granularity_probe.py > $out/granularity.jsonl 2> $out/granularity.err
run 900 python -u bench.py > $out/bench.log 2>&1
