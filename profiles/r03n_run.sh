#!/bin/bash
# r03n: the host path on dla_host_reduce_launch / _join (ABI v9: the round streams on a library
# thread while the caller allocates and clones the result under the interpreter lock; the last
# chunk's unpack spread over threads): the GPU suite (C demo included), smoke, host phases per
# config, the per-config host-inclusive table twice; then a north-star tile-size sweep.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03n
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
run 300 env DLA_HOST_REDUCE_STATS=1 python -u profiles/host_phases_probe.py "configs[2],configs[3'],configs[4]" > $out/phases.log 2>&1
run 300 python -u bench.py --host-configs-only > $out/hostcfg1.log 2>&1
run 300 python -u bench.py --host-configs-only > $out/hostcfg2.log 2>&1
run 300 python -u profiles/ab_r03_kernels.py --shapes ns --stages "" --ns-tiles 32768,65536,262144,1048576 > $out/ns_tiles.log 2>&1
