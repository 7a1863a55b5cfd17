# A/B in one process: the previous commit's library (libdlagg_prev.so) vs the current build,
# default launch (auto kernel pick), on the given shapes (args: "peers params dtype" ...).
set -e
L=decentralized-learning_amd/lib
for cfg in "$@"; do
  set -- $cfg
  echo "== peers=$1 params=$2 dtype=$3"
  timeout -k 10 120 python bench.py --sweep --no-ceilings --libs $L/libdlagg_prev.so,$L/libdlagg.so --peers $1 --params $2 --dtype $3 --sweep-cfgs "0,0,0,0"
done
