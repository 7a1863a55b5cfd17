#!/bin/bash
# r03ar: the north star at 32 KiB tiles (the PeerSlab's tile for <= 8 rows) capped at W = 14 vs 15,
# three alternating processes each.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ar
mkdir -p $out
for r in 1 2 3; do
  for w in 14 15; do
    DLA_VEC_WGS_PER_CU=$w timeout -k 10 300 python -u profiles/ab_r03_kernels.py --shapes ns,b8 --stages "" --rounds 5 \
      --ns-tiles 32768 > $out/w${w}_r${r}.log 2>&1 || exit $?
  done
done
