#!/bin/bash
# r04w: address-translation counters of the many-tensor table kernel (16 / 128 google_speech ResNet-34
# models in separate allocations) against the north star's tile-interleaved slab kernel: is the table
# kernel's gap to the flat slab (131 vs 102 us on the same bytes) UTCL1 misses?  Two rocprofv3 --pmc passes
# (4 TCP + 2 GRBM counters at most each), summarised by profiles/pmc_summary.py.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04w
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
P1=TCP_UTCL1_REQUEST_sum,TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum,TCP_UTCL1_STALL_MULTI_MISS_sum
P2=TCP_UTCL1_SERIALIZATION_STALL_sum,TCP_UTCL1_THRASHING_STALL_sum,TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum,TCP_UTCL1_STALL_INFLIGHT_MAX_sum,GRBM_GUI_ACTIVE,GRBM_UTCL2_BUSY
run 180 rocprofv3 --pmc $P1 --output-format csv -d $out/pmc_t1 -o run -- python3 profiles/pmc_driver.py r34x16,r34x128,ns --reps 20 > $out/pmc_t1.log 2>&1
run 180 rocprofv3 --pmc $P2 --output-format csv -d $out/pmc_t2 -o run -- python3 profiles/pmc_driver.py r34x16,r34x128,ns --reps 20 > $out/pmc_t2.log 2>&1
run 60 python3 profiles/pmc_summary.py $out/pmc_tlb_summary.json $out/pmc_t1 $out/pmc_t2
rm -rf $out/pmc_t1 $out/pmc_t2
