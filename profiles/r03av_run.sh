#!/bin/bash
# r03av: the final round-3 tree (native library unchanged since r03ap): GPU suite, smoke, bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03av
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1
