# A/B: runtime-peer big tiles (variant 32) vs the default pick, for the many-peer BASELINE shares
set -e
for cfg in "32 1690046 f32" "64 1233086 f32" "16 21296355 f32" "128 2662045 bf16" "8 25000000 f32" "4 25000000 f32" "12 10000000 f32"; do
  set -- $cfg
  echo "== peers=$1 params=$2 dtype=$3"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype $3 --sweep-cfgs "0,0,0,0;32,0,0,0;4,1,0,64"
done
