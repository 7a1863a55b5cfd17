#!/bin/bash
# r04d (a second box): the occupancy-cap rule against round 3's table (tuning build, DLA_VEC_CAP_TABLE=1),
# the table kernel's 8-byte against 16-byte loads (A/B build lib/ab/libdlagg_vw.so), the device-module
# round's host-time breakdown, and configs[2]'s host round phases (tuning build, DLA_HOST_REDUCE_STATS=1).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04d
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
run 300 python -u profiles/r04_multi_pipe_ab.py --lib decentralized-learning_amd/lib/ab/libdlagg_vw.so --knob DLA_MULTI_VW --values 2,4 > $out/multi_vw_ab.log 2>&1
run 300 python -u profiles/r04_device_round_probe.py > $out/device_round.log 2>&1
run 300 env ACCDFL_AMD_TUNING=1 DLA_HOST_REDUCE_STATS=1 python -u profiles/host_phases_probe.py "configs[2],configs[3']" > $out/host_phases.log 2>&1
