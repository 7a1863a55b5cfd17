"""Round 5: the host time before a device round's first launch (profiles/r05n: the launch call returns
0.084 ms after FedAvg.aggregate starts for 16 google_speech ResNet-34 models, of which the walk is 30 us
and the launch call 17 us).  Wraps the steps FedAvg.aggregate takes for device modules with timestamps
(relative to the call) and prints their medians over 200 calls."""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

import bench  # noqa: E402
from accdfl_amd import _lib  # noqa: E402
from accdfl_amd.core import wsum as _wsum  # noqa: E402
from accdfl_amd.core.gradient_aggregation import fedavg as fa  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    models, _ = bench._device_layout_models("google_speech_resnet34", n, torch.bfloat16, dev)
    w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
    marks = []
    t0 = [0.0]

    def wrap(mod, name):
        real = getattr(mod, name)

        def f(*a, **k):
            marks.append((name + ">", time.perf_counter() - t0[0]))
            r = real(*a, **k)
            marks.append((name + "<", time.perf_counter() - t0[0]))
            return r
        setattr(mod, name, f)

    for mod, name in ((fa, "_device_layout"), (fa, "_native_layout"), (fa, "_device_round"), (fa, "_flat_plan"),
                      (_wsum, "wsum_multi_ptrs"), (_lib, "wsum_multi_table_ptrs"), (fa, "_seed_buffers"),
                      (fa, "_clone_value")):
        wrap(mod, name)
    fa._wsum.wsum_multi_ptrs = _wsum.wsum_multi_ptrs
    import gc

    for gc_on in (True, False):
        if not gc_on:
            gc.disable()
        run(models, w, marks, t0, n, gc_on)
    gc.enable()


def run(models, w, marks, t0, n, gc_on):
    rows = []
    for it in range(220):
        marks.clear()
        torch.cuda.synchronize()
        t0[0] = time.perf_counter()
        fa.FedAvg.aggregate(models, w)
        ret = time.perf_counter() - t0[0]
        torch.cuda.synchronize()
        if it >= 20:
            rows.append([(k, v) for k, v in marks] + [("return", ret)])
    keys = [k for k, _ in rows[0]]
    med = [(k, round(statistics.median(r[i][1] for r in rows) * 1e6, 1)) for i, k in enumerate(keys)]
    print(json.dumps({"peers": n, "gc_enabled": gc_on, "us_from_call": med}), flush=True)


if __name__ == "__main__":
    main()
