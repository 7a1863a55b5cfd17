#!/bin/bash
# r03ai: do 8 or 16 peers per round plus an occupancy cap generalise to large many-peer passes?
# 32 x 10 M, 48 x 6 M, 64 x 4.93 M, 64 x 8 M f32 (4 KiB tiles) and configs[4] whole: variants 8 / 12
# against the default at W = none / 8 / 10 / 12 (DLA_VEC_WGS_PER_CU applies to every tree leg).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ai
mkdir -p $out
for w in 0 8 10 12; do
  DLA_VEC_WGS_PER_CU=$w timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes p32x10,p48x6,c3p,p64x8,c4whole \
    --stages "" --rounds 4 --variants 8,12 > $out/w${w}.log 2>&1 || exit $?
done
