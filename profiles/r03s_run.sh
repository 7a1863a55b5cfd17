#!/bin/bash
# r03s: egress straight from HBM (DeviceModelManager.aggregate_serialized through wire.DeviceSource):
# the wire / DFL / call-site GPU tests, then the DFL round probe twice (aggregate + serialize_model vs
# aggregate_serialized).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03s
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "wire or dfl or call_site or serialized or ingress" > $out/tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 300 python -u profiles/dfl_round_probe.py > $out/dfl_r${r}.log 2>&1 || exit $?
done
