#!/bin/bash
# r03i: host path A/B, interleaved on one box: streaming-store packs (DLA_COPY_NT=1/0) x copy threads
# (DLA_COPY_THREADS=8/16), FedAvg.aggregate on CPU modules of configs[2] / configs[3'] (phases probe);
# then the host-path parity tests.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03i
mkdir -p $out
for r in 1 2; do
  for nt in 1 0; do
    for th in 8 16; do
      DLA_COPY_NT=$nt DLA_COPY_THREADS=$th timeout -k 10 200 python -u profiles/host_phases_probe.py "configs[2],configs[3']" \
        > $out/ab_nt${nt}_th${th}_r${r}.log 2>&1 || exit 1
    done
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "host or native or layouts or call_sites or dfl or fedavg_cpu or result_memory or staging" > $out/tests.log 2>&1
