#!/bin/bash
# r02: tile-interleaved slab (dla_wsum_slab_tiled) vs the row-major default, interleaved A/B.
set -e
OUT=${OUT:-gpurun_out/ab_tiled.log}
: > "$OUT"
run() {
  echo "== $1 peers x $2 $3" >> "$OUT"
  timeout -k 10 150 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype $3 \
    --tile-bytes 1024,4096,16384 >> "$OUT" 2>&1
}
run 128 2662045 bf16
run 128 21296355 bf16
run 64 1233086 f32
run 32 1690046 f32
run 16 21296355 bf16
run 8 25000000 f32
run 128 85354 f32
