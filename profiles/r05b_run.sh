#!/bin/bash
# r05b: round-5 tree on the GPU: the new tests first (mixed-dtype parity through dla_wsum_mixed, ABI v13;
# bf16 / 8-rank gloo sharding with the HIP reducer), then the whole -m gpu suite, smoke, and the default
# N=1 bench (its cpu_baseline leg now checks the headline's output against the oracle port).
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
run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
