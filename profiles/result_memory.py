"""r02: where the host-inclusive round's time goes with a pageable vs a page-locked result.

FedAvg.aggregate (8 CPU modules x 25 M fp32, the reference call sites' situation) in each
result-memory mode of core/host_memory.py, and the pieces apart: faulting in a fresh 100 MB
pageable tensor, a 100 MB D2H into fresh pageable / reused pageable / page-locked memory.
Run on the GPU box (order of the modes alternates between rounds)."""
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


def t_ms(fn, reps=4):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e3, 2)


def main():
    n, p = 8, 25_000_000
    g = torch.Generator().manual_seed(2000)
    models = []
    for _ in range(n):
        m = nn.Module()
        m.w = nn.Parameter(torch.randn(p, generator=g) * 0.05)
        models.append(m)
    w = [1.0 / n] * n
    dev = torch.empty(p, device="cuda").normal_()
    reused = torch.empty(p)
    reused.zero_()
    pinned = torch.empty(p, pin_memory=True)
    res = {"threads": torch.get_num_threads()}
    res["fault_in_fresh_100MB_ms"] = t_ms(lambda: torch.empty(p).fill_(0))
    res["d2h_fresh_pageable_ms"] = t_ms(lambda: torch.empty(p).copy_(dev))
    res["d2h_reused_pageable_ms"] = t_ms(lambda: reused.copy_(dev))
    res["d2h_pinned_ms"] = t_ms(lambda: pinned.copy_(dev, non_blocking=True))
    print(json.dumps(res), flush=True)
    agg = {}
    for rnd in range(3):
        modes = ("pooled", "pinned", "pageable") if rnd % 2 == 0 else ("pageable", "pinned", "pooled")
        for mode in modes:
            host_memory.set_result_memory(mode)
            agg.setdefault(mode, []).append(t_ms(lambda: FedAvg.aggregate(models, w)))
    for mode, v in agg.items():
        print(json.dumps({"mode": mode, "ms": v, "GB/s": round((n + 1) * p * 4 / (min(v) / 1e3) / 1e9, 1)}))


if __name__ == "__main__":
    main()
