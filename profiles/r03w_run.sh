#!/bin/bash
# r03w: finer occupancy sweep of the tiled vector kernel (DLA_VEC_LDS_PAD bytes of dynamic LDS per
# workgroup -> workgroups per CU), every f32 / bf16 shape the bench and the PeerSlab run, each process
# timing the tree build with the pad against the base build without it, interleaved.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03w
mkdir -p $out
for pad in 0 8704 9472 10240 11008 12032 13312; do
  DLA_VEC_LDS_PAD=$pad timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes ns,ns4,ns16,b16,c2,c3p \
    --stages "" --rounds 5 > $out/pad${pad}.log 2>&1 || exit $?
done
