#!/bin/bash
# r03an: configs[4]'s per-GPU share (128 x 2 662 045 bf16) and configs[3']'s bucket (64 x 1 233 086 f32)
# with 8 / 16 KiB tiles beside the default 4 KiB, plus 16 peers per round, at W = none / 12.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03an
mkdir -p $out
for w in 0 12; do
  DLA_VEC_WGS_PER_CU=$w timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes c4share,c3b --stages "" \
    --rounds 5 --ns-tiles 8192,16384 --variants 12 > $out/w${w}.log 2>&1 || exit $?
done
timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes c4share,c3b --stages "" --rounds 5 \
  --ns-tiles 8192,16384 --variants 12 > $out/policy.log 2>&1
