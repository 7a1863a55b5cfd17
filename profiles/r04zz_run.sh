#!/bin/bash
# r04zz: the final round-4 tree (after the native-clone switch's rename): GPU suite + smoke.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04zz
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
