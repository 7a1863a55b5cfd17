#!/bin/bash
# r06q: the egress fill's copy threads and D2H chunk size (tuning build knobs DLA_COPY_THREADS,
# ACCDFL_AMD_EGRESS_CHUNK_MB), profiles/r06_egress_split.py per setting, NUMA-bound like the bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06q
mkdir -p $out
for cfg in "8 32" "16 32" "8 8" "16 8" "16 4" "8 32"; do
  set -- $cfg
  echo "{\"copy_threads\": $1, \"chunk_mb\": $2}" >> $out/sweep.jsonl
  ACCDFL_AMD_TUNING=1 DLA_COPY_THREADS=$1 ACCDFL_AMD_EGRESS_CHUNK_MB=$2 timeout -k 10 150 \
    python -u profiles/r06_egress_split.py --numa-bind >> $out/sweep.jsonl 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc" >> $out/sweep.jsonl; exit $rc; fi
done
