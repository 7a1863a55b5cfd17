#!/bin/bash
# r06a: the round-6 tree with the world-4/8 RCCL cases (skipped on one GPU), the table-device fix and the
# ADVICE r05 wire / manager fixes: GPU suite + smoke, the default N=1 bench, and the 4-rank gloo rehearsal
# (configs[3]'s world size) on the one GPU.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06a
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
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
run 900 python -u bench.py --gpus 4 --dist-backend gloo --steps 20 --warmup 5 > $out/gloo4.log 2>&1
