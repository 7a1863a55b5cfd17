#!/bin/bash
# r03ah: 8 separate fp32 peers over >= 256 MiB through the row-major vector kernel capped at 16
# workgroups per CU (replacing the big tile), bf16 8-peer rows capped alike: the GPU suite + smoke,
# the A/B (tree policy vs base) with separate-buffer legs, the default bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ah
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
run 400 python -u profiles/ab_r03_kernels.py --shapes ns,b8,ns16,b16 --stages "" --rounds 5 --rows 9 > $out/ab.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
