#!/bin/bash
# r04f: host rounds reading the packed page-locked rows with the vector-per-lane kernel against the
# staging DMAs (tuning build DLA_HOST_STAGE_DMA=1), four alternating processes each, then the GPU suite.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04f
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
for i in 1 2 3 4; do
  run 300 python -u bench.py --host-configs-only > $out/hostcfg_read_$i.log 2>&1
  run 300 env ACCDFL_AMD_TUNING=1 DLA_HOST_STAGE_DMA=1 python -u bench.py --host-configs-only > $out/hostcfg_dma_$i.log 2>&1
done
run 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
