# Wide (variant 8) vs 16-byte stream (variant 4, 64x1) around the auto-selection threshold.
set -e
for cfg in "16 262144 f32" "32 262144 f32" "32 524288 f32" "64 524288 f32" "128 524288 f32" "32 1048576 f32" "64 1048576 f32" \
           "128 1048576 f32" "64 1233086 f32" "128 665511 bf16" "128 1331022 bf16" "128 2662045 bf16" "32 1690046 f32" \
           "128 21339 bf16" "128 21339 f32" "64 21339 f32" "200 85354 f32"; do
  set -- $cfg
  echo "== peers=$1 params=$2 dtype=$3"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype $3 --sweep-cfgs "8,0,0,0;4,1,0,64"
done
