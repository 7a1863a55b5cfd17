#!/bin/bash
# r05p: the occupancy cap on the strong-split buckets (tuning build, DLA_VEC_WGS_PER_CU), interleaved.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${R05P_OUT:-r05p}
mkdir -p $out
export ACCDFL_AMD_TUNING=1
for rep in 1 2; do
  for c in rule 0 14; do
    if [ $c = rule ]; then unset DLA_VEC_WGS_PER_CU; else export DLA_VEC_WGS_PER_CU=$c; fi
    timeout -k 10 120 python -u profiles/r05_share_cap_probe.py >> $out/cap.jsonl 2>> $out/cap.err || exit $?
  done
done
