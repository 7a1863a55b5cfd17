#!/bin/bash
# r04e: the reduce reading packed page-locked staging rows across PCIe (no staging DMAs) and the native
# buffer copies of the device round: GPU suite + smoke, the default bench, the device-round breakdown,
# and host-inclusive configs with / without the staging DMAs (tuning build DLA_HOST_STAGE_DMA=1),
# three alternating processes each.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04e
mkdir -p $out
run() {
  local t=$1; shift
  echo "$(date +%T) start: $*" >> $out/steps.log
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$(date +%T) rc=$rc: $*" >> $out/steps.log
  case $rc in 124|137|134|139) exit $rc;; esac
  return 0
}
run 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
run 300 python -u profiles/r04_device_round_probe.py > $out/device_round.log 2>&1
for i in 1 2 3; do
  run 300 python -u bench.py --host-configs-only > $out/hostcfg_read_$i.log 2>&1
  run 300 env ACCDFL_AMD_TUNING=1 DLA_HOST_STAGE_DMA=1 python -u bench.py --host-configs-only > $out/hostcfg_dma_$i.log 2>&1
done
