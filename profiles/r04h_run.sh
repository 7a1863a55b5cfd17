#!/bin/bash
# r04h: pageable PeerSlab sources through device chunks (the wire_ingress regression), buffer gathers for
# CPU deep copies: GPU suite + smoke, the default N=1 bench, the DFL phase split.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04h
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
run 300 python -u profiles/r04_dfl_phases.py > $out/dfl_phases.log 2>&1
