#!/bin/bash
# Round 5: the new dfl_round_layout leg (configs[4]'s ResNet-34 through EVA blocks) alone, then the
# default bench line with it.
set -o pipefail
mkdir -p gpurun_out/r05ai
timeout -k 10 300 python -u -c "
import json, torch, bench
print(json.dumps(bench.dfl_round_layout('google_speech_resnet34', 16, torch.bfloat16, torch.device('cuda', 0))))
print(json.dumps(bench.dfl_round_layout('cifar10_resnet8', 64, torch.float32, torch.device('cuda', 0))))
" > gpurun_out/r05ai/dfl_layout.log 2>&1 || { tail -30 gpurun_out/r05ai/dfl_layout.log; exit 1; }
cat gpurun_out/r05ai/dfl_layout.log | grep -v amdgpu.ids
timeout -k 10 900 python -u bench.py > gpurun_out/r05ai/bench.log 2>&1; rc=$?
tail -c 400 gpurun_out/r05ai/bench.log; exit $rc
