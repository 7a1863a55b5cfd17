#!/bin/bash
# r04s3: the small-round bound at 48 MiB (from r04s2's crossover): GPU suite + smoke, the crossover probe
# again (its "small" leg is now the default routing), the default N=1 bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04s3
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && \
timeout -k 10 400 python -u profiles/r04_small_large_ab.py > $out/small_large_ab.jsonl 2> $out/small_large_ab.err && \
timeout -k 10 900 python -u bench.py > $out/bench.log 2>&1
