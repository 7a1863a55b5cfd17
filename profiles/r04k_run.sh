#!/bin/bash
# r04k: host rounds with 8 (product default) against 12 and 16 pack threads (tuning build DLA_COPY_THREADS),
# three alternating processes each (configs[2] pageable was pack-bound on slower hosts: r04j 5.05 ms).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04k
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
  run 300 python -u bench.py --host-configs-only > $out/hostcfg_t8_$i.log 2>&1
  run 300 env ACCDFL_AMD_TUNING=1 DLA_COPY_THREADS=12 python -u bench.py --host-configs-only > $out/hostcfg_t12_$i.log 2>&1
  run 300 env ACCDFL_AMD_TUNING=1 DLA_COPY_THREADS=16 python -u bench.py --host-configs-only > $out/hostcfg_t16_$i.log 2>&1
done
