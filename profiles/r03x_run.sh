#!/bin/bash
# r03x: the tiled vector kernel capped at W workgroups per CU (DLA_VEC_WGS_PER_CU; dynamic LDS sized
# so that exactly W fit), W = none / 10-24, on the north star and the other few-peer shapes; each
# process times the tree build capped against the base build uncapped, interleaved.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03x
mkdir -p $out
for w in 0 10 12 13 14 15 16 18 20 24; do
  DLA_VEC_WGS_PER_CU=$w timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes ns,ns16,b16,b8,ns4,ns2 \
    --stages "" --rounds 5 > $out/w${w}.log 2>&1 || exit $?
done
