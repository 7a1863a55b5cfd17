#!/bin/bash
# r05h: counters behind the table kernel's gap to the flat slab: per-channel TCC read
# requests and busy cycles (TCC_EA0_RDREQ / TCC_BUSY per instance x XCC), read latency, and address
# translation (UTCL1 misses, TA stalls on TC, UTCL2 busy) for 16 / 128 ResNet-34 bf16 device modules
# (wsum_multi_vec_kernel) against the tiled slab of the same bytes (wsum_vec_kernel).  One pass per run.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05h
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
S=r34x16,r34flat16,r34x128,c4whole
run 120 rocprofv3 --pmc TCC_EA0_RDREQ TCC_BUSY GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_chan -o run -- python3 profiles/pmc_driver.py $S --reps 10 > $out/pmc_chan.log 2>&1
run 120 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_lat -o run -- python3 profiles/pmc_driver.py $S --reps 10 > $out/pmc_lat.log 2>&1
run 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_tlb -o run -- python3 profiles/pmc_driver.py $S --reps 10 > $out/pmc_tlb.log 2>&1
run 60 python3 profiles/r05_pmc_channels.py $out/pmc_channels_summary.json $out/pmc_chan $out/pmc_lat $out/pmc_tlb > $out/summary.log 2>&1
