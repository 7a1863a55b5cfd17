#!/bin/bash
# r03z: the occupancy-cap policy in the library (vec_wgs_cap): the whole GPU suite + smoke, the default
# N=1 bench, the rocprofv3 trace + FETCH / WRITE passes of the headline, and the tree (policy) against
# the base build (uncapped) on every tiled shape.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03z
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
run 1000 bash profiles/collect.sh r03z --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-small
cp gpurun_out/prof_r03z/summary/* gpurun_out/prof_r03z/trace.log $out/ 2>/dev/null
rm -rf gpurun_out/prof_r03z
run 600 python -u profiles/ab_r03_kernels.py --shapes ns,b8,ns16,b16,ns12,ns4,ns6,ns2,c2,c3p,c4share --stages "" --rounds 5 > $out/ab.log 2>&1
