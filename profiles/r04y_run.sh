#!/bin/bash
# r04y: the egress chunk ramp (wire._egress_chunks: a small first D2H and a small last copy-out) against
# uniform 32 MiB chunks, 100 MB from HBM into serialize_model bytes, four interleaved rounds of fresh
# processes (profiles/r04_egress_probe.py), then the DFL round leg of the bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04y
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
for i in 1 2 3 4; do
  for r in 0 1; do
    run 120 env ACCDFL_AMD_EGRESS_RAMP=$r python -u profiles/r04_egress_probe.py >> $out/egress.jsonl 2>> $out/egress.err
  done
done
run 300 python -u -m pytest tests/test_gpu_dfl_round.py -x -q --timeout 120 --timeout-method thread > $out/dfl_tests.log 2>&1
