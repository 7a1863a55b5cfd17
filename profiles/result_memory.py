"""r02: host-inclusive FedAvg.aggregate (8 CPU modules x 25 M fp32, the reference call sites'
situation) in each result-memory mode of core/host_memory.py, and the small GNLeNet round
(unaffected: it scatters into the result on the host).  Run on the GPU box."""
import json
import os
import statistics
import sys
import time

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
from accdfl_amd.core import host_memory  # noqa: E402
from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg  # noqa: E402


def main():
    n, p = 8, 25_000_000
    g = torch.Generator().manual_seed(2000)
    models = []
    for _ in range(n):
        m = nn.Module()
        m.w = nn.Parameter(torch.randn(p, generator=g) * 0.05)
        models.append(m)
    w = [1.0 / n] * n
    res = {}
    for rnd in range(3):
        for mode in ("pinned", "pageable"):
            host_memory.set_result_memory(mode)
            FedAvg.aggregate(models, w)
            ts = []
            for _ in range(4):
                t0 = time.perf_counter()
                out = FedAvg.aggregate(models, w)
                ts.append(time.perf_counter() - t0)
                del out
            res.setdefault(mode, []).append(statistics.median(ts) * 1e3)
    for mode, v in res.items():
        print(json.dumps({"mode": mode, "ms": [round(x, 2) for x in v],
                          "GB/s": round((n + 1) * p * 4 / (min(v) / 1e3) / 1e9, 1)}))


if __name__ == "__main__":
    main()
