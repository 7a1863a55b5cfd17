#!/bin/bash
# Round 5: the large host-round fuzz (rounds above the small-round bound through the chunked host paths).
set -o pipefail
mkdir -p gpurun_out/r05ag
timeout -k 10 600 python -u -m pytest tests/test_fuzz_fedavg.py -m gpu -k large -v --timeout 200 --timeout-method thread -rf \
  > gpurun_out/r05ag/fuzz_large.log 2>&1; rc=$?
tail -40 gpurun_out/r05ag/fuzz_large.log; exit $rc
