#!/bin/bash
# r06z: the final round-6 tree's evidence (after the worker-thread parameter blocks): the whole GPU suite + smoke, the default N=1 bench, the rocprofv3 kernel
# trace + FETCH / WRITE passes of the headline (profiles/collect.sh), and the 4- and 8-rank gloo rehearsals
# (configs[3]'s and configs[4]'s world sizes) on the one GPU.
# Plus the host/GPU split of a 16-model device round (profiles/r06_device_round_split.py).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06z
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
run 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rs > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 900 python -u bench.py > $out/bench.log 2>&1
run 1000 bash profiles/collect.sh r06z --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-small
cp gpurun_out/prof_r06z/summary/* gpurun_out/prof_r06z/trace.log $out/ 2>/dev/null
rm -rf gpurun_out/prof_r06z
run 120 python -u profiles/r06_device_round_split.py > $out/device_round_split.jsonl 2>&1
run 120 python -u profiles/r06_device_round_split.py --tree > $out/device_round_split_tree.jsonl 2>&1
run 200 python -u profiles/r06_clone_probe.py > $out/clone.jsonl 2>&1
run 300 python -u profiles/r06_async_blocks_probe.py > $out/async_blocks.jsonl 2>&1
run 900 python -u bench.py --gpus 4 --dist-backend gloo --steps 20 --warmup 5 > $out/gloo4.log 2>&1
run 900 python -u bench.py --gpus 8 --dist-backend gloo --steps 20 --warmup 5 > $out/gloo8.log 2>&1
