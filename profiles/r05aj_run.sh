#!/bin/bash
# Round 5: the many-tensor DFL ingress probe (profiles/r05_dfl_layout_probe.py).
set -o pipefail
mkdir -p gpurun_out/r05aj
timeout -k 10 300 python -u profiles/r05_dfl_layout_probe.py > gpurun_out/r05aj/probe.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05aj/probe.log | head -60; exit $rc
