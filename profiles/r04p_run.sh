#!/bin/bash
# r04p: the device round's host work step by step, the group schedules' launch timelines and their
# interleaved end-to-end A/B (profiles/r04_device_round_split.py).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04p
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
run 600 python -u profiles/r04_device_round_split.py > $out/device_split.log 2>&1
