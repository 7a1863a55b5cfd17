#!/bin/bash
# r03at: balanced persistent grid for the tiled vector kernel (DLA_VEC_PERSIST = X workgroups per CU,
# each striding over the same number of 64-vector blocks) against one workgroup per block (X = 0) and
# the saved pre-change build ("base"), on the north star, configs[4]'s share and whole model and
# configs[3']'s bucket.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03at
mkdir -p $out
for x in 0 16 12 8 14; do
  DLA_VEC_PERSIST=$x timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes ns,c4share,c4whole,c3b \
    --stages "" --rounds 5 > $out/x${x}.log 2>&1 || exit $?
done
