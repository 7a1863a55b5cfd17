#!/bin/bash
# Collect the rocprofv3 evidence behind bench.py's roofline numbers (run on the GPU box):
#   1. kernel trace + stats of the bench command (average launch duration per kernel)
#   2. FETCH_SIZE pass and 3. WRITE_SIZE pass (separate --pmc passes, as the
#      MI355X guide's HBM section prescribes; FETCH_SIZE is doubled for gfx950 16-B streams)
# then summarises them into profiles/<round>_*.  Usage: bash profiles/collect.sh r01 [bench args]
set -euo pipefail
ROUND=${1:-r01}; shift || true
ARGS="$*"  # default: the exact bench.py command the driver runs
OUT=gpurun_out/prof_$ROUND
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
python3 profiles/summarize.py "$OUT" "$ROUND" $ARGS
# summaries land in $OUT/summary/ (merged back by gpurun); copy them into profiles/ to commit
