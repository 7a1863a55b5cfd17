# A/B: stream (4) vs big tile (16) vs balanced big tile (17: partial last round spread over
# one round of 64-chunk segment workgroups), at shapes whose last round of tiles is partial.
set -e
for cfg in "8 21300000" "8 22500000" "8 26000000" "16 14000000" "16 21296355" "32 6250000" "8 25000000" "16 12500000"; do
  set -- $cfg
  echo "== peers=$1 params=$2 f32"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype f32 --sweep-cfgs "4,1,0,64;16,0,0,0;17,0,0,0"
done
