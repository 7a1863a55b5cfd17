#!/bin/bash
# r03au: configs[4]'s share and whole model (128 bf16 peers) as passes of 64 / 43 / 32 peers over the
# tiled slab (DLA_TILED_PASS_PEERS; out carries the bf16 running sum between passes, bit-exact) against
# the single 128-peer pass; the saved build ("base") in every process.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03au
mkdir -p $out
for p in 0 64 43 32; do
  DLA_TILED_PASS_PEERS=$p timeout -k 10 400 python -u profiles/ab_r03_kernels.py --shapes c4share,c4whole \
    --stages "" --rounds 5 > $out/p${p}.log 2>&1 || exit $?
done
