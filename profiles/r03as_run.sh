#!/bin/bash
# r03as: configs[4]'s per-GPU share (128 x 2 662 045 bf16) over 1 / 2 / 32 / 64 KiB tiles beside the
# default 4 KiB (8 and 16 KiB are in r03an), default policy, two processes.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03as
mkdir -p $out
for r in 1 2; do
  timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes c4share --stages "" --rounds 5 \
    --ns-tiles 1024,2048,32768,65536 > $out/r${r}.log 2>&1 || exit $?
done
