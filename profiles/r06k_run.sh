#!/bin/bash
# r06k: the result-allocation probe with the buffer copy split in its halves; smoke and the wire tests on the
# rebuilt walk extension.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06k
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
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 300 python -u profiles/r06_result_alloc_probe.py > $out/result_alloc.jsonl 2> $out/result_alloc.err
run 600 python -u -m pytest tests/test_wire.py tests/test_wire_scan.py tests/test_gpu_dfl_round.py -m gpu -q --timeout 300 --timeout-method thread -rs > $out/gpu_tests.log 2>&1
