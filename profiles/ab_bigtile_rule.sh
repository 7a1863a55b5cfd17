# Check of the big-tile rule (use_bigtile): default launch (0) vs the 64 x 1 stream (4) vs the
# big tile (16) vs the balanced big tile (17), at shapes on both sides of the rule.
set -e
for cfg in "8 25000000" "8 21300000" "8 26000000" "8 3400000" "16 12500000" "16 14000000" "16 21296355" "32 4110000" "32 6250000"; do
  set -- $cfg
  echo "== peers=$1 params=$2 f32"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype f32 --sweep-cfgs "0,0,0,0;4,1,0,64;16,0,0,0;17,0,0,0"
done
