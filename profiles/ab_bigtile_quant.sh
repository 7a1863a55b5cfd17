# Wave-quantization probe: big-tile (variant 16) vs default at sizes whose big-tile count
# (n_chunks / 1024) falls just under / just over a multiple of the resident-wave slots.
set -e
for cfg in "8 21300000" "8 22500000" "8 25000000" "8 26000000" "16 12500000" "16 14000000" "16 16000000" "16 21296355" "16 24500000"; do
  set -- $cfg
  echo "== peers=$1 params=$2 f32"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype f32 --sweep-cfgs "4,1,0,64;16,0,0,0"
done
