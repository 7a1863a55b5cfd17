#!/bin/bash
# r06c: the allocation-granularity A/B of the table kernel — 16 / 128 google_speech
# ResNet-34 bf16 device models with one caching-allocator block per parameter (today) against one
# allocation per model (256-byte aligned views): HIP-event times (profiles/r06_granularity_probe.py), then
# the r05h translation and latency counter passes over the same launches (profiles/pmc_driver.py).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06c
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
run 300 python -u profiles/r06_granularity_probe.py > $out/granularity.jsonl 2> $out/granularity.err
# one rocprofv3 run per shape and pass: the separate and contiguous layouts launch the same kernel with the
# same grid, so their dispatches are told apart by directory
for S in r34x16 r34x16c r34x128 r34x128c; do
  run 180 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d $out/tlb_$S -o run -- python3 profiles/pmc_driver.py $S --reps 10 > $out/tlb_$S.log 2>&1
  run 180 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $out/lat_$S -o run -- python3 profiles/pmc_driver.py $S --reps 10 > $out/lat_$S.log 2>&1
done
run 60 python3 profiles/r05_pmc_channels.py $out/pmc_granularity_summary.json $out/tlb_r34x16 $out/tlb_r34x16c $out/tlb_r34x128 $out/tlb_r34x128c $out/lat_r34x16 $out/lat_r34x16c $out/lat_r34x128 $out/lat_r34x128c > $out/summary.log 2>&1
