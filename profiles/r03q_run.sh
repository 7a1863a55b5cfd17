#!/bin/bash
# r03q: the DFL round with the EVA-block gather into page-locked ingress buffers on streaming stores
# (dla_host_copy_batch_ex, DLA_COPY_STREAMING) against plain stores (ACCDFL_AMD_INGRESS_NT=0),
# interleaved, three times; then the wire / DFL / ingress GPU tests.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03q
mkdir -p $out
for r in 1 2 3; do
  for nt in 1 0; do
    ACCDFL_AMD_INGRESS_NT=$nt timeout -k 10 300 python -u profiles/dfl_round_probe.py > $out/dfl_nt${nt}_r${r}.log 2>&1 || exit $?
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "wire or dfl or ingress or serialized or c_abi or copy_batch" > $out/tests.log 2>&1
