#!/bin/bash
# r05ak: the round-5 tree with the dfl_round_layout leg and the block-reader change: GPU suite + smoke, the default N=1 bench, the rocprofv3 kernel
# trace + FETCH / WRITE passes of the headline (profiles/collect.sh), and the 8-rank gloo rehearsal.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05ak
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
run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
run 1000 bash profiles/collect.sh r05ak --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-small
cp gpurun_out/prof_r05ak/summary/* gpurun_out/prof_r05ak/trace.log $out/ 2>/dev/null
rm -rf gpurun_out/prof_r05ak
run 900 python -u bench.py --gpus 8 --dist-backend gloo --steps 20 --warmup 5 > $out/gloo8.log 2>&1
run 300 python -u profiles/r05_table_probe.py > $out/table_probe.jsonl 2> $out/table_probe.err
run 400 python -u profiles/r04_device_round_split.py > $out/device_split.log 2>&1
