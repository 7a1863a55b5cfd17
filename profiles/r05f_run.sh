#!/bin/bash
# r05f: the table-upload policy and the ring's amortised events in the product build: the multi-table
# GPU tests, the probe (policy, no tuning knobs), bench.py's device_module_configs rows, and a kernel +
# copy trace of the 16 x ResNet-34 bf16 table reduce.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r05f
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
run 500 python -u -m pytest tests/test_gpu_parity.py tests/test_center_copy_layouts.py -m gpu -x -v -k "multi_table or device_modules or mixed or record_stream or reference_trees" --timeout 200 --timeout-method thread > $out/table_tests.log 2>&1
run 300 python -u profiles/r05_table_probe.py > $out/probe.jsonl 2> $out/probe.err
run 300 python -u profiles/r05_table_probe.py >> $out/probe.jsonl 2>> $out/probe.err
run 300 python -u bench.py --device-configs-only > $out/device_configs.log 2>&1
run 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/trace -o run -- python -u profiles/r05_table_probe.py "16 peers" > $out/trace.log 2>&1
