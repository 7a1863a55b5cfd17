#!/bin/bash
# r02: interleaved A/B of the many-peer kernels (run on the GPU box from the repo root):
# 0 = default pick, 8 = word-per-lane (dword), 9 = dwordx2 x 32 peers, 10 = dwordx4 x 16,
# 11 = dwordx4 x 32, 12 = dwordx2 x 16, 4,1,0,64 = 16-byte stream.
set -e
OUT=${OUT:-gpurun_out/ab_vec.log}
: > "$OUT"
run() {
  echo "== $1 peers x $2 $3" >> "$OUT"
  timeout -k 10 150 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype $3 \
    --sweep-cfgs "0,0,0,0;8,0,0,0;9,0,0,0;10,0,0,0;11,0,0,0;12,0,0,0;4,1,0,64" >> "$OUT" 2>&1
}
run 128 2662045 bf16
run 128 21296355 bf16
run 128 665511 bf16
run 64 1233086 f32
run 32 1690046 f32
run 128 85354 f32
run 64 21339 f32
run 16 21296355 bf16
