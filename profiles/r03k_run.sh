#!/bin/bash
# r03k: host path after the fast parameter walk: phases of FedAvg.aggregate on CPU modules
# (configs[2], [3'], [4]) and the per-config host-inclusive table (3 runs).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03k
mkdir -p $out
timeout -k 10 300 python -u profiles/host_phases_probe.py "configs[2],configs[3'],configs[4]" > $out/phases.log 2>&1 &&
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --host-configs-only > $out/hostcfg_r${r}.log 2>&1 || exit 1
done
