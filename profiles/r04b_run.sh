#!/bin/bash
# r04b: the second box of the two-box A/Bs — the occupancy-cap rule against round 3's table (tuning build with
# DLA_VEC_CAP_TABLE=1) and the pipelined table kernel against the one-block kernel; plus the NS trace.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04b
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
run 400 env DLA_VEC_CAP_TABLE=1 python -u profiles/ab_r03_kernels.py --base decentralized-learning_amd/lib/libdlagg_tuning.so --auto-tile --no-ldsdma --shapes ns,ns4,n9,ns12,ns16,b8,b16,ns2,ns6,c4share --rounds 5 --reps 20 > $out/cap_ab.log 2>&1
run 300 python -u profiles/r04_multi_pipe_ab.py > $out/multi_pipe_ab.log 2>&1
