#!/bin/bash
# r03a: the round-3 tests added so far, then the multi-rank bench rehearsed on the one-GPU box
# (4 gloo ranks sharing GPU 0: every N > 1 leg with its parity flag), then the default N=1 bench.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03a
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "freed or footprint or small_round_waits or ingress_slot or tiled_slab_dirichlet or tiled_4k" \
  > $out/new_tests.log 2>&1 &&
timeout -k 10 900 python -u bench.py --gpus 4 --dist-backend gloo --steps 20 --warmup 5 --leg-timeout 400 \
  > $out/gloo4.log 2>&1 &&
timeout -k 10 900 python -u bench.py > $out/bench.log 2>&1
