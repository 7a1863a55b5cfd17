#!/bin/bash
# r06h: native scan with the blob-prefix fast path and native row_layout: the wire / manager GPU tests, the
# ingress phase split (NUMA-bound this time), the default bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06h
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
run 600 python -u -m pytest tests/test_wire.py tests/test_gpu_dfl_round.py tests/test_fuzz_model_manager.py tests/test_call_sites.py tests/test_wire_scan.py -m gpu -q --timeout 300 --timeout-method thread -rs > $out/gpu_tests.log 2>&1
run 300 python -u profiles/r06_ingress_split.py --numa-bind > $out/ingress_split.jsonl 2> $out/ingress_split.err
run 900 python -u bench.py > $out/bench.log 2>&1
