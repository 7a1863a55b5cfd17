#!/bin/bash
# r03u: dla_host_reduce's first-chunk ramp (DLA_HOST_RAMP = 2 / 4 / 8 / 16: the first chunk is 1/k of
# a chunk, then doubling) on configs[2] and configs[3'] as CPU modules (host phases probe), three
# interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03u
mkdir -p $out
for r in 1 2 3; do
  for k in 2 4 8 16; do
    DLA_HOST_RAMP=$k timeout -k 10 200 python -u profiles/host_phases_probe.py "configs[2],configs[3']" \
      > $out/ramp${k}_r${r}.log 2>&1 || exit $?
  done
done
