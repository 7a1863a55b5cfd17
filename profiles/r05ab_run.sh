#!/bin/bash
# Round 5: the table kernel's workgroup -> XCD order (translation-bound, profiles/r05h).  Workgroups are
# dealt to the 8 XCDs round-robin, so every XCD touches every page of every peer; DLA_TABLE_XCD_RUN=R
# (tuning build) hands each XCD runs of R consecutive workgroups instead (R = 1: the product order; the
# whole-eighth remap of profiles/r05j lost).  Each R in its own process, interleaved twice.
# Ran against a tuning build whose wsum_multi_vec_kernel remapped blockIdx.x in super-blocks of 8 R
# (XCD x of the round-robin deal taking logical workgroups x R .. x R + R - 1); R = 1 won on every
# layout, so the remap was not kept and DLA_TABLE_XCD_RUN is no longer read.
set -o pipefail
export TMPDIR=/tmp ACCDFL_AMD_TUNING=1
mkdir -p gpurun_out/r05ab
for rep in 1 2; do
  for r in 1 2 4 16 64 256; do
    echo "{\"xcd_run\": $r, \"rep\": $rep}" >> gpurun_out/r05ab/xcd_run.jsonl
    DLA_TABLE_XCD_RUN=$r timeout -k 10 150 python -u profiles/r05_table_probe.py \
      ResNet-34 ResNet-8 FEMNIST >> gpurun_out/r05ab/xcd_run.jsonl 2>> gpurun_out/r05ab/err.log || exit $?
    echo "rep $rep run $r done"
  done
done
