#!/bin/bash
# r03v: occupancy cap of the tiled vector kernel through dynamic LDS per workgroup (DLA_VEC_LDS_PAD):
# the north star (32 VGPRs: 8 waves per SIMD uncapped) and configs[4]'s share (100 VGPRs: 4), each
# process timing the tree build with the pad against the r03 base build without it, interleaved.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03v
mkdir -p $out
for pad in 0 4096 6144 8192 10240 16384; do
  DLA_VEC_LDS_PAD=$pad timeout -k 10 300 python -u profiles/ab_r03_kernels.py --shapes ns,c4share --stages "" \
    > $out/pad${pad}.log 2>&1 || exit $?
done
