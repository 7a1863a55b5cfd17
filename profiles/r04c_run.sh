#!/bin/bash
# r04c: native EVA block bookkeeping + native result-parameter views (walk.cpp), then: GPU suite + smoke,
# the default bench, the DFL phase split, the table kernel's counters (16 / 128 x ResNet-34 bf16 device
# modules) beside the north star's, the occupancy-cap rule A/B and the pipelined table-kernel A/B.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04c
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
run 300 python -u profiles/r04_dfl_phases.py > $out/dfl_phases.log 2>&1
run 400 env DLA_VEC_CAP_TABLE=1 python -u profiles/ab_r03_kernels.py --base decentralized-learning_amd/lib/libdlagg_tuning.so --auto-tile --no-ldsdma --shapes ns,ns4,n9,ns12,ns16,b8,b16,ns2,ns6,c4share --rounds 5 --reps 20 > $out/cap_ab.log 2>&1
run 300 python -u profiles/r04_multi_pipe_ab.py > $out/multi_pipe_ab.log 2>&1
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LEVEL_WAVES SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_CYCLES"
run 180 rocprofv3 --pmc $P1 --output-format csv -d $out/pmc_p1 -o run -- python3 profiles/pmc_driver.py r34x16,r34x128,ns --reps 20 > $out/pmc_p1.log 2>&1
run 180 rocprofv3 --pmc $P2 --output-format csv -d $out/pmc_p2 -o run -- python3 profiles/pmc_driver.py r34x16,r34x128,ns --reps 20 > $out/pmc_p2.log 2>&1
run 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- python3 profiles/pmc_driver.py r34x16,r34x128,ns --reps 20 > $out/pmc_fetch.log 2>&1
run 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- python3 profiles/pmc_driver.py r34x16,r34x128,ns --reps 20 > $out/pmc_write.log 2>&1
run 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/pmc_trace -o run -- python3 profiles/pmc_driver.py r34x16,r34x128,ns --reps 20 > $out/pmc_trace.log 2>&1
run 60 python3 profiles/pmc_summary.py $out/pmc_summary.json $out/pmc_p1 $out/pmc_p2 $out/pmc_fetch $out/pmc_write
rm -rf $out/pmc_p1 $out/pmc_p2 $out/pmc_fetch $out/pmc_write
