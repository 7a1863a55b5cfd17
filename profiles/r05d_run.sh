#!/bin/bash
# r05d: table-upload modes 0-4 (tuning build, DLA_TABLE_COPY) with single-call and end-to-end latency,
# then kernel + copy traces of modes 1, 3 and 4 on 16 x ResNet-34 bf16.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05d
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
export ACCDFL_AMD_TUNING=1
for m in 0 1 2 3 4 0 1 2 3 4; do
  DLA_TABLE_COPY=$m run 300 python -u profiles/r05_table_probe.py >> $out/modes.jsonl 2>> $out/modes.err
done
for m in 1 3 4; do
  DLA_TABLE_COPY=$m run 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/trace_m$m -o run -- python -u profiles/r05_table_probe.py "16 peers" > $out/trace_m$m.log 2>&1
done
