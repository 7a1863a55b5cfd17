#!/bin/bash
# r03m: (1) the counters this pool's rocprofv3 offers; (2) the GPU suite on the one-instruction bf16
# rounding build; (3) interleaved A/B: tree vs the r03 base build on the tiled slab (NS, configs[4]
# share / whole, 16 x 21.3 M bf16) and the LDS-DMA north-star probe; (4) SQ counter passes
#  for the north star and configs[4]'s share, base and tree builds; (5) FETCH /
# WRITE passes and a kernel trace of the tree build; (6) host-path phases with the deferred-output
# native call (ABI v9) and the PCIe ceilings of the box.  A step that times out, aborts or faults
# ends the script; other failures are logged and the next step runs.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03m
mkdir -p $out
base=decentralized-learning_amd/lib/ab/libdlagg_r03base.so
run() {
  local t=$1; shift
  echo "$(date +%T) start: $*" >> $out/steps.log
  timeout -k 10 "$t" "$@"
  local rc=$?
  echo "$(date +%T) rc=$rc: $*" >> $out/steps.log
  case $rc in 124|137|134|139) exit $rc;; esac
  return 0
}
run 60 rocprofv3 -L > $out/counters_avail.txt 2>&1
run 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
run 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
run 400 python -u profiles/ab_r03_kernels.py > $out/ab.log 2>&1
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_LEVEL_WAVES SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_CYCLES"
for lib in base tree; do
  la=""; [ $lib = base ] && la="--lib $base"
  run 120 rocprofv3 --pmc $P1 --output-format csv -d $out/pmc_${lib}_p1 -o run -- python3 profiles/pmc_driver.py ns,c4share $la > $out/pmc_${lib}_p1.log 2>&1
  run 120 rocprofv3 --pmc $P2 --output-format csv -d $out/pmc_${lib}_p2 -o run -- python3 profiles/pmc_driver.py ns,c4share $la > $out/pmc_${lib}_p2.log 2>&1
done
run 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_tree_fetch -o run -- python3 profiles/pmc_driver.py ns,c4share > $out/pmc_tree_fetch.log 2>&1
run 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_tree_write -o run -- python3 profiles/pmc_driver.py ns,c4share > $out/pmc_tree_write.log 2>&1
run 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_tree -o run -- python3 profiles/pmc_driver.py ns,c4share,c4whole > $out/trace_tree.log 2>&1
run 300 env DLA_HOST_REDUCE_STATS=1 python -u profiles/host_phases_probe.py "configs[2],configs[3'],configs[4]" > $out/phases.log 2>&1
run 120 python -u profiles/pcie_probe.py 256 > $out/pcie.log 2>&1
