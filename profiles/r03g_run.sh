#!/bin/bash
# r03g: dla_host_reduce with a ramped chunk schedule (1/4, 1/2, then full chunks; dense per-chunk
# pitch, one contiguous H2D per chunk) and _large_round cloning the result module while the native
# call runs: host-path parity tests, the phases probe, the per-config host-inclusive table.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03g
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "host or native or layouts or call_sites or dfl or fedavg_cpu or result_memory or staging" > $out/tests.log 2>&1 &&
DLA_HOST_REDUCE_STATS=1 timeout -k 10 300 python -u profiles/host_phases_probe.py "configs[2],configs[3'],configs[4]" \
  > $out/phases.log 2>&1 &&
timeout -k 10 300 python -u bench.py --host-configs-only > $out/hostcfg.log 2>&1
