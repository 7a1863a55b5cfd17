#!/bin/bash
# r04i: PeerSlab keeps page-locked sources until their copies finish; host-memory reads of the small-round
# path on the vector kernel too: GPU suite + smoke, then small rounds vector kernel / shape-chosen kernel,
# three alternating processes each.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04i
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
for i in 1 2 3; do
  run 200 python -u profiles/r04_small_rounds.py >> $out/small_vec.log 2>&1
  run 200 env ACCDFL_AMD_TUNING=1 DLA_HOST_AUTO_KERNEL=1 python -u profiles/r04_small_rounds.py >> $out/small_auto.log 2>&1
done
run 300 python -u bench.py --host-configs-only > $out/hostcfg.log 2>&1
