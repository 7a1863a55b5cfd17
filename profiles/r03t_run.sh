#!/bin/bash
# r03t: aggregate_serialized's copy-out from HBM: bounce chunk 8 / 32 / 64 MiB x plain / streaming
# stores into the fresh payload, interleaved twice (DFL round probe: aggregate_serialized_ms).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03t
mkdir -p $out
for r in 1 2; do
  for ch in 8 32 64; do
    for nt in 0 1; do
      ACCDFL_AMD_EGRESS_CHUNK_MB=$ch ACCDFL_AMD_EGRESS_NT=$nt timeout -k 10 300 python -u profiles/dfl_round_probe.py \
        > $out/dfl_ch${ch}_nt${nt}_r${r}.log 2>&1 || exit $?
    done
  done
done
