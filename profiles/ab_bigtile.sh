# A/B: 16-byte stream (variant 4, 64 x 1) vs the peer-major big-tile kernel (variant 16) for
# <= 8 peers, to place the auto-selection rule (use_bigtile in csrc/dlagg.hip).
set -e
for cfg in "8 25000000 f32" "7 25000000 f32" "6 25000000 f32" "5 25000000 f32" "3 25000000 f32" "1 25000000 f32" \
           "8 3000000 f32" "8 2097152 f32" "8 1500000 f32" "8 12500000 f64" "4 12500000 f64" "2 12500000 f64" \
           "1 12500000 f64" "8 1048576 f64"; do
  set -- $cfg
  echo "== peers=$1 params=$2 dtype=$3"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype $3 --sweep-cfgs "4,1,0,64;16,0,0,0"
done
