#!/bin/bash
# r03f: where dla_host_reduce's time goes on configs[2] (FEMNIST, 32 CPU models) and configs[3']
# (ResNet-8, 64 CPU models): per-call phase times (DLA_HOST_REDUCE_STATS=1), rank bound to the GPU's
# NUMA node as bench.py binds it.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03f
mkdir -p $out
PROBE_BIND=gpu DLA_HOST_REDUCE_STATS=1 timeout -k 10 300 python -u profiles/host_reduce_probe.py "configs[2],configs[3']" \
  > $out/probe.log 2>&1
