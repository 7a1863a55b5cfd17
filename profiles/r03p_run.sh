#!/bin/bash
# r03p: the DFL aggregator round (bench dfl_round: ingress of 8 EVA-block messages of a 25 M fp32 model,
# average, serialize) with the gather's copy threads at 8 / 12 / 16, twice, interleaved; the per-peer
# split of the ingress.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03p
mkdir -p $out
for r in 1 2; do
  for th in 8 12 16; do
    DLA_COPY_THREADS=$th timeout -k 10 300 python -u profiles/dfl_round_probe.py > $out/dfl_th${th}_r${r}.log 2>&1 || exit $?
  done
done
