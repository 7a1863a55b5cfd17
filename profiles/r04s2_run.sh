#!/bin/bash
# r04s2: the small-round / pipelined-round crossover for CPU models re-measured on the round-4 host paths
# (profiles/r04_small_large_ab.py).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04s2
mkdir -p $out
timeout -k 10 400 python -u profiles/r04_small_large_ab.py > $out/small_large_ab.jsonl 2> $out/small_large_ab.err
