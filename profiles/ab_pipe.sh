set -e
L=decentralized-learning_amd/lib
for cfg in "64 21339 f32" "64 1233086 f32" "32 1690046 f32" "128 2662045 bf16" "16 85354 f32" "128 21296355 bf16"; do
  set -- $cfg
  echo "== peers=$1 params=$2 dtype=$3"
  timeout -k 10 200 python bench.py --sweep --no-ceilings --libs $L/libdlagg_base.so,$L/libdlagg.so --peers $1 --params $2 --dtype $3 --sweep-cfgs "4,1,0,64"
done
