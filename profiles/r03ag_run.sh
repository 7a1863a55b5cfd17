#!/bin/bash
# r03ag: peers as separate row-major buffers (device-resident modules of one big tensor): the default
# kernel (peer-major big tile for fp32 8 / 16 peers) against the row-major vector kernel (variant 9)
# with the occupancy cap applied to it (DLA_VEC_CAP_ROWS=1) at W = none / 10-16.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ag
mkdir -p $out
for w in 0 10 12 14 16; do
  DLA_VEC_CAP_ROWS=1 DLA_VEC_WGS_PER_CU=$w timeout -k 10 300 python -u profiles/ab_r03_kernels.py --shapes ns,ns16,b8 \
    --stages "" --rounds 4 --rows 9 > $out/w${w}.log 2>&1 || exit $?
done
