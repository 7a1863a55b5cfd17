#!/bin/bash
# r03ac: the occupancy cap for the peer counts the policy does not list yet (3, 5, 7, 9-11, 13-15 peers
# x 25 M f32): W = none / 10-28 workgroups per CU, tree capped vs base uncapped in each process.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ac
mkdir -p $out
for w in 0 10 12 14 16 18 20 24 28; do
  DLA_VEC_WGS_PER_CU=$w timeout -k 10 400 python -u profiles/ab_r03_kernels.py \
    --shapes n3,n5,n7,n9,n10,n11,n13,n14,n15 --stages "" --rounds 4 > $out/w${w}.log 2>&1 || exit $?
done
