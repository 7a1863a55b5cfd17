#!/bin/bash
# r03al: north star with 32 KiB tiles at W = 12-18 workgroups per CU (tree 16 KiB default leg beside it).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03al
mkdir -p $out
for w in 12 14 15 16 18; do
  DLA_VEC_WGS_PER_CU=$w timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes ns --stages "" --rounds 5 \
    --ns-tiles 32768 > $out/w${w}.log 2>&1 || exit $?
done
