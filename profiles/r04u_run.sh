#!/bin/bash
# r04u: result tensors with a storage each over one allocation (walk.cpp alias_of: pickles like deepcopy),
# CPU results' parameters over one allocation, the module tree cloned natively module by module: GPU
# suite + smoke, the device-round split and schedule A/B, the device-round probe, the default N=1 bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04u
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
run 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
run 400 python -u profiles/r04_device_round_split.py > $out/device_split.log 2>&1
run 300 python -u profiles/r04_device_round_probe.py > $out/device_round.log 2>&1
