#!/bin/bash
# r03l: after the native host walk: the whole GPU suite + smoke, the host-path phases, the
# device-resident module rounds, the default N=1 bench, and the 4-rank gloo rehearsal of the N>1 legs.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03l
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 300 python -u profiles/host_phases_probe.py "configs[2],configs[3'],configs[4]" > $out/phases.log 2>&1 &&
timeout -k 10 300 python -u bench.py --device-configs-only > $out/device_configs.log 2>&1 &&
timeout -k 10 900 python -u bench.py > $out/bench.log 2>&1 &&
timeout -k 10 900 python -u bench.py --gpus 4 --dist-backend gloo --steps 20 --warmup 5 > $out/gloo4.log 2>&1
