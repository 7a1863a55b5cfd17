#!/bin/bash
# r03ak: the north star's tile size re-measured under the occupancy cap (tree: 16 KiB default plus
# 4 / 32 / 64 / 256 KiB re-tiled copies of the same peers; base: uncapped, 16 KiB), twice.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03ak
mkdir -p $out
for r in 1 2; do
  timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes ns,b8 --stages "" --rounds 5 \
    --ns-tiles 4096,32768,65536,262144 > $out/tiles_r${r}.log 2>&1 || exit $?
done
