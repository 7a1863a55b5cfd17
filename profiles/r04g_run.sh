#!/bin/bash
# r04g: the round-4 tree so far end to end — GPU suite + smoke, the default N=1 bench (the driver's command),
# the rocprofv3 kernel trace + FETCH / WRITE passes of the headline (profiles/collect.sh), the device-round
# breakdown, and the 4-rank gloo rehearsal of the N>1 legs (strong_headline included).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04g
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
run 1000 bash profiles/collect.sh r04g --steps 20 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-small
cp gpurun_out/prof_r04g/summary/* gpurun_out/prof_r04g/trace.log $out/ 2>/dev/null
rm -rf gpurun_out/prof_r04g
run 300 python -u profiles/r04_device_round_probe.py > $out/device_round.log 2>&1
run 900 python -u bench.py --gpus 4 --dist-backend gloo --steps 20 --warmup 5 > $out/gloo4.log 2>&1
# the table kernel under an occupancy cap of W workgroups per CU (0 = none, the product's choice): A/B build
run 300 python -u profiles/r04_multi_pipe_ab.py --lib decentralized-learning_amd/lib/ab/libdlagg_wgs.so --knob DLA_MULTI_WGS --values 0,12,16,20,24 --shapes r34x16,r34x32,r8x16,r8x32,femx32 > $out/multi_wgs_ab.log 2>&1
# the table kernel with narrower fold rounds (8 peers for 9-32-peer passes, 16 above): A/B build
run 300 python -u profiles/r04_multi_pipe_ab.py --lib decentralized-learning_amd/lib/ab/libdlagg_g.so --knob DLA_MULTI_G --values 0,8 --shapes r34x16,r34x32,r8x16,r8x32,femx32 > $out/multi_g8_ab.log 2>&1
run 300 python -u profiles/r04_multi_pipe_ab.py --lib decentralized-learning_amd/lib/ab/libdlagg_g.so --knob DLA_MULTI_G --values 0,16 --shapes r34x128,r8x64 > $out/multi_g16_ab.log 2>&1
