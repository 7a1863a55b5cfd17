"""r04: where a device-resident module round's host time goes (FedAvg.aggregate on 16
google_speech ResNet-34 models in HBM took 2.0 ms end to end against a 0.13 ms reduce; round 4's target
is the reduce + 0.15 ms).  For 16 and 128 ResNet-34 bf16 models (bench.py's device_module_configs
layout): the end-to-end median, the median of each step of fedavg._device_round timed alone, and a
cProfile of 50 aggregates (top entries by own time).
Usage on the GPU box: python profiles/r04_device_round_probe.py -> JSON lines + the profile text."""
import cProfile
import io
import json
import os
import pstats
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch import nn  # noqa: E402

from accdfl_amd import _lib  # noqa: E402
from accdfl_amd.core.gradient_aggregation import fedavg as fa  # noqa: E402


def med_ms(fn, reps=30, sync=True):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e3, 4)


def main():
    dev = torch.device("cuda", 0)
    for n in (16, 128):
        models, p = bench._device_layout_models("google_speech_resnet34", n, torch.bfloat16, dev)
        w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
        row = {"peers": n, "end_to_end_ms": med_ms(lambda: fa.FedAvg.aggregate(models, w))}
        row["host_layout_ms"] = med_ms(lambda: fa._host_layout(models), sync=False)
        row["device_layout_ms"] = med_ms(lambda: fa._device_layout(models), sync=False)
        layout = fa._device_layout(models)
        row["device_round_no_sync_ms"] = med_ms(lambda: fa._device_round(models, w, layout), sync=False)
        mod = _lib.walk_module()
        row["tensors_walk_ms"] = med_ms(lambda: mod.tensors(models[0], fa._PLAIN_SET), sync=False)
        p0, b0 = mod.tensors(models[0], fa._PLAIN_SET)
        row["seed_buffers_ms"] = med_ms(lambda: fa._seed_buffers(b0, {}), sync=False)
        memo = {}
        fa._seed_buffers(b0, memo)
        row["clone_tree_ms"] = med_ms(lambda: fa._clone_value(models[0], dict(memo)), sync=False)
        print(json.dumps(row), flush=True)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(50):
            fa.FedAvg.aggregate(models, w)
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(s.getvalue(), flush=True)
        del models
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
