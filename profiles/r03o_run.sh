#!/bin/bash
# r03o: launched host rounds on persistent per-device library workers (no thread creation or HIP
# first-call set-up per round): host-path tests, host phases per config (with the launch->start /
# run / end->join split), the per-config host-inclusive table three times.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03o
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
run 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "host or native or layouts or call_sites or dfl or fedavg_cpu or result_memory or staging or deferred or abandon or c_abi" > $out/tests.log 2>&1
run 300 env DLA_HOST_REDUCE_STATS=1 python -u profiles/host_phases_probe.py "configs[2],configs[3'],configs[4]" > $out/phases.log 2>&1
for r in 1 2 3; do
  run 300 python -u bench.py --host-configs-only > $out/hostcfg$r.log 2>&1
done
