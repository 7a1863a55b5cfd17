#!/bin/bash
# Round 5: table-kernel shape A/B (translation-bound, profiles/r05h): dwords per lane x runs per
# workgroup, interleaved twice, each shape in its own process (the knobs are read once).
# Ran against a tuning build whose wsum_multi_vec_kernel took VW (dwords per lane) and CH (runs of 64
# vectors per workgroup, one after the other) as template arguments, chosen by DLA_TABLE_VW /
# DLA_TABLE_CH, and whose r05_table_probe.py echoed them as "shape" in each line.  Every variant lost
# to the product's VW = 2, CH = 1, so the knobs were not kept: this script now runs
# the product shape each time.
set -o pipefail
export TMPDIR=/tmp ACCDFL_AMD_TUNING=1
mkdir -p gpurun_out/r05aa
for rep in 1 2; do
  for shape in "2 1 0" "4 1 0" "2 4 0" "2 8 0" "4 4 0"; do
    set -- $shape
    DLA_TABLE_VW=$1 DLA_TABLE_CH=$2 DLA_TABLE_WGS=$3 timeout -k 10 150 python -u profiles/r05_table_probe.py \
      ResNet-34 ResNet-8 FEMNIST >> gpurun_out/r05aa/shape.jsonl 2>> gpurun_out/r05aa/err.log || exit $?
    echo "rep $rep shape $shape done"
  done
done
