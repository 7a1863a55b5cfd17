#!/bin/bash
# r02: vec-kernel tail rounds split into G/2, G/4, ..., 1 (libdlagg.so) against a partial last
# round that reloads the last peer into the spare slots (libdlagg_nosplit.so: the A/B build kept
# that round behind a VEC_TAIL_SPLIT=0 switch, removed once the split won), tiled slab and
# separate buffers, peer counts that leave a tail.  Usage: bash profiles/ab_tail.sh
set -o pipefail
run() { timeout -k 10 200 python -u bench.py --sweep --no-ceilings "$@" 2>&1 | grep -v amdgpu.ids; }
for lib in libdlagg.so libdlagg_nosplit.so; do
  export DLAGG_LIB=$PWD/decentralized-learning_amd/lib/$lib
  echo "## $lib"
  for shape in "2 25000000 f32 16384" "4 25000000 f32 16384" "6 25000000 f32 16384" "12 11173962 f32 16384" \
               "20 5000000 f32 4096" "48 1233086 f32 4096" "100 2662045 bf16 4096" "3 50000000 bf16 16384"; do
    set -- $shape
    echo "# peers $1 params $2 $3 tile $4"
    run --peers $1 --params $2 --dtype $3 --tile-bytes $4 --sweep-cfgs 0 || exit 1
  done
done
