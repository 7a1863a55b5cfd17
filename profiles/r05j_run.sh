#!/bin/bash
# r05j: (1) the table kernel with XCD-contiguous workgroups (tuning build, DLA_MULTI_XCD=1) against the
# dispatcher's round-robin order, interleaved, on every device layout; (2) the product tree: the table
# policy's probe + trace, the GPU suite, smoke and the default bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05j
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
for x in 0 1 0 1; do
  ACCDFL_AMD_TUNING=1 DLA_MULTI_XCD=$x run 300 python -u profiles/r05_table_probe.py >> $out/xcd.jsonl 2>> $out/xcd.err
  echo "{\"xcd_remap\": $x}" >> $out/xcd.jsonl
done
run 300 python -u profiles/r05_table_probe.py > $out/probe.jsonl 2> $out/probe.err
run 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/trace -o run -- python -u profiles/r05_table_probe.py "16 peers" > $out/trace.log 2>&1
run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
