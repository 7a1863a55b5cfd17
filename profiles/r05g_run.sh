#!/bin/bash
# r05g: what is left between two table-reduce kernels: the policy (hipStreamQuery + side copy) against
# forced side copies with no stream query (DLA_TABLE_COPY=3) and no upload at all (=5, diagnostic: the
# back-to-back kernels alone), with kernel traces of 16 x ResNet-34 bf16.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05g
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
for m in -1 3 5; do
  DLA_TABLE_COPY=$m run 300 python -u profiles/r05_table_probe.py "16 peers" "ResNet-8" "128 peers" >> $out/modes.jsonl 2>> $out/modes.err
  DLA_TABLE_COPY=$m run 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/trace_m$m -o run -- python -u profiles/r05_table_probe.py "16 peers" > $out/trace_m$m.log 2>&1
done
