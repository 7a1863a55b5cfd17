#!/bin/bash
# r04y: the egress chunk ramp (wire._egress_chunks: a small first D2H and a small last copy-out) against
# uniform 32 MiB chunks, 100 MB from HBM into serialize_model bytes, four interleaved rounds of fresh
# processes (profiles/r04_egress_probe.py); then, on the final tree, the GPU suite + smoke and the default
# N=1 bench.
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
run 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
