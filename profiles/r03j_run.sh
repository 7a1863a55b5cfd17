#!/bin/bash
# r03j: dla_host_reduce without the cross-queue wait in front of every chunk's DMA (when the reduce that
# last read the device buffer has already finished) — interleaved A/B against always waiting
# (DLA_HOST_WAIT_ALWAYS=1), phases of FedAvg.aggregate on CPU modules of configs[2] / configs[3'];
# then the whole GPU suite and smoke (variants 10/11 removed, multi-table search simplified).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03j
mkdir -p $out
for r in 1 2 3; do
  timeout -k 10 200 python -u profiles/host_phases_probe.py "configs[2],configs[3']" > $out/ab_skip_r${r}.log 2>&1 &&
  DLA_HOST_WAIT_ALWAYS=1 timeout -k 10 200 python -u profiles/host_phases_probe.py "configs[2],configs[3']" \
    > $out/ab_always_r${r}.log 2>&1 || exit 1
done
DLA_HOST_REDUCE_STATS=1 timeout -k 10 200 python -u profiles/host_phases_probe.py "configs[2],configs[3']" > $out/stats.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
