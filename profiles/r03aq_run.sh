#!/bin/bash
# r03aq: under the occupancy cap, plain output stores for the north star (variant 21 / 28: 8 peers per
# round with plain stores) against the sc1 default; 8 x 50 M bf16 alike; twice.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03aq
mkdir -p $out
for r in 1 2; do
  timeout -k 10 300 python -u profiles/ab_r03_kernels.py --shapes ns,b8,ns16 --stages "" --rounds 5 --variants 21,28 \
    > $out/stores_r${r}.log 2>&1 || exit $?
done
