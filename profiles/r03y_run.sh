#!/bin/bash
# r03y: finer workgroups-per-CU caps: 16-peer passes (W 6-10), 12 and 6 peers, 4 peers (W 24-30), the
# north star again (W 14, 15); tree capped vs base uncapped in each process.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03y
mkdir -p $out
for w in 0 6 7 8 9 10 11 12 14 15 18 21 24 26 28 30; do
  DLA_VEC_WGS_PER_CU=$w timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes ns,ns16,b16,ns12,ns6,ns4 \
    --stages "" --rounds 5 > $out/w${w}.log 2>&1 || exit $?
done
