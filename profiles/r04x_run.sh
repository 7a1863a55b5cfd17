#!/bin/bash
# r04x: the egress copy-out's chunk size (wire._EGRESS_CHUNK): 100 MB from HBM into serialize_model bytes at
# 4, 8, 16 and 32 MiB chunks bound to the GPU's NUMA node and 32 MiB unbound, three interleaved rounds of fresh
# processes (profiles/r04_egress_probe.py).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04x
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
for i in 1 2 3; do
  for mb in 4 8 16 32; do
    run 120 env ACCDFL_AMD_EGRESS_CHUNK_MB=$mb python -u profiles/r04_egress_probe.py >> $out/egress.jsonl 2>> $out/egress.err
  done
  run 120 env EGRESS_NO_BIND=1 python -u profiles/r04_egress_probe.py >> $out/egress.jsonl 2>> $out/egress.err
done
