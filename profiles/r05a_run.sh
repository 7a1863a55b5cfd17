#!/bin/bash
# r05a: the round-4 tree as it stands, first 8-rank rehearsal: bench.py --gpus 8 over gloo (8 ranks
# sharing the box's one GPU), every leg incl. the strong configs[4] bf16 split, then the default bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05a
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
run 900 python -u bench.py --gpus 8 --dist-backend gloo --steps 20 --warmup 5 > $out/gloo8.log 2>&1
run 600 python -u bench.py > $out/bench.log 2>&1
