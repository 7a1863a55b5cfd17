#!/bin/bash
# r03aa: many-peer passes (32-128 peers) with fewer loads in flight per lane and an occupancy cap:
# launch variants 8 / 28 (8 peers per round, sc1 / plain stores) and 12 (16) against the default (32)
# at W = none / 8-20 workgroups per CU (DLA_VEC_WGS_PER_CU), configs[4]'s share and whole model,
# configs[3']'s whole model and bucket; the base build uncapped in every process.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03aa
mkdir -p $out
for w in 0 8 10 12 14 16 20; do
  DLA_VEC_WGS_PER_CU=$w timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes c4share,c4whole,c3p,c3b \
    --stages "" --rounds 5 --variants 8,28,12 > $out/w${w}.log 2>&1 || exit $?
done
