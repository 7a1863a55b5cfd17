#!/bin/bash
# r06p: evidence on the tree with the two-step result parameters: the whole GPU suite, smoke, the default
# N=1 bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06p
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
run 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rs > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
