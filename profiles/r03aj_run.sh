#!/bin/bash
# r03aj: the many-peer cap in the library (>= 32 peers over >= 1 GiB: 16 peers per round, 8 at 64
# peers, 8 workgroups per CU): the GPU suite, then tree (policy) vs base on the large many-peer
# shapes and the ones the policy leaves alone.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03aj
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u profiles/ab_r03_kernels.py --shapes p32x10,p48x6,c3p,p64x8,c4whole,c4share,c3b,c2,ns,b16 \
  --stages "" --rounds 5 > $out/ab.log 2>&1
