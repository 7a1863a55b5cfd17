# A/B in one process: the r01 session-2 library (libdlagg_base.so: 16-byte stream, one-lane
# ragged tail) against the current build (auto: wide kernel for small many-peer shares,
# lane-parallel tail), default launch shape, across the BASELINE per-GPU shares and odd sizes.
set -e
L=decentralized-learning_amd/lib
for cfg in "64 21339 f32" "64 21336 f32" "8 85354 f32" "4 116 f32" "64 85354 f32" "128 85354 f32" "16 85354 f32" \
           "32 1690046 f32" "64 1233086 f32" "128 2662045 bf16" "128 21339 bf16" "8 25000001 f32" "8 25000000 f32"; do
  set -- $cfg
  echo "== peers=$1 params=$2 dtype=$3"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --libs $L/libdlagg_base.so,$L/libdlagg.so --peers $1 --params $2 --dtype $3 --sweep-cfgs "0,0,0,0"
done
