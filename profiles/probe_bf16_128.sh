# Why is 128 peers x 21 339 bf16 slow (36-43 us for 5.5 MB) when 128 x 85 354 f32 (43 MB) takes 13 us?
set -e
for cfg in "128 21339 bf16" "128 21340 bf16" "128 21376 bf16" "128 21343 bf16" "128 21339 f32" "128 10670 f32" "64 21339 bf16" "128 21339 f16" "32 21339 bf16" "128 85354 f32"; do
  set -- $cfg
  echo "== peers=$1 params=$2 dtype=$3"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --peers $1 --params $2 --dtype $3 --sweep-cfgs "8,0,0,0;4,1,0,64"
done
