#!/bin/bash
# r05i: the table upload with the host-side busy estimate (no hipStreamQuery): probe + trace of the
# product policy, the GPU suite, smoke and the default bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05i
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
run 300 python -u profiles/r05_table_probe.py > $out/probe.jsonl 2> $out/probe.err
run 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/trace -o run -- python -u profiles/r05_table_probe.py "16 peers" > $out/trace.log 2>&1
run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
