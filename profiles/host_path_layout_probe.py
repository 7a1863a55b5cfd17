"""native (dla_host_reduce) vs pipelined (one H2D per tensor per peer per chunk) host paths on the
reference layouts at few and many peers (the GL merge is N=2, a DFL round N=8..64): median us of
FedAvg.aggregate on CPU modules, NUMA-bound.  Decides which large-round path a round takes."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

from accdfl_amd.core.gradient_aggregation import fedavg as F  # noqa: E402
from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402

print(json.dumps({"numa_node_bound": bind_to_gpu_node()}), flush=True)


def med(fn, reps=9):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


for lay, ns in (("femnist_cnn", (2, 4, 8, 32)), ("cifar10_resnet8", (2, 3, 4, 8, 64)), ("gnlenet", (8, 64))):
    for n in ns:
        models, p = bench._layout_models(lay, n, torch.float32, False)
        w = [1.0 / n] * n
        r = {"layout": lay, "n": n, "params": p, "tensors": len(list(models[0].parameters())),
             "input_MB": round(n * p * 4 / 1e6, 1)}
        small = n * p * 4 < (256 << 20)
        default = F._SMALL_ROW_BYTES, F._SMALL_ROUND_BYTES
        for mode in ("native", "pipelined", "small", "native", "pipelined", "small"):
            if mode == "small":
                if not small:
                    continue
                F._SMALL_ROW_BYTES = F._SMALL_ROUND_BYTES = 1 << 40
            else:
                F._SMALL_ROW_BYTES = F._SMALL_ROUND_BYTES = 0
                F.set_host_path(mode)
            r.setdefault(mode + "_us", []).append(med(lambda: F.FedAvg.aggregate(models, w)))
            F._SMALL_ROW_BYTES, F._SMALL_ROUND_BYTES = default
        F.set_host_path("native")
        r["default_us"] = med(lambda: F.FedAvg.aggregate(models, w))
        print(json.dumps(r), flush=True)
        del models
