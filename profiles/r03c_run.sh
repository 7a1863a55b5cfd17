#!/bin/bash
# r03c: the device-resident module rounds (FedAvg.aggregate on HBM modules of the reference layouts,
# dla_wsum_multi_table vs the per-tensor path vs the flat PeerSlab), plain and under a kernel trace.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03c
mkdir -p $out
timeout -k 10 600 python -u bench.py --device-configs-only > $out/device_configs.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- \
  python3 -u bench.py --device-configs-only > $out/trace.log 2>&1
