"""r02: FedAvg.aggregate of CPU-resident models, small-round path (dla_host_round_*: pack into
page-locked rows, the kernel reads them across PCIe) against the large-round paths — native
(dla_host_reduce: packed chunks, one DMA per chunk) and pipelined (chunked H2D straight from the
parameters overlapping the D2H) — forced by _SMALL_ROW_BYTES / _SMALL_ROUND_BYTES, per input size.
The process is bound to the GPU's NUMA node first (as bench.py does)."""
import json
import os
import statistics
import sys
import time

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
from accdfl_amd.core.gradient_aggregation import fedavg as F  # noqa: E402


def med(fn, reps):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def main():
    from accdfl_amd.core.host_memory import bind_to_gpu_node

    print(json.dumps({"numa_node_bound": bind_to_gpu_node()}), flush=True)
    default = F._SMALL_ROW_BYTES, F._SMALL_ROUND_BYTES
    for n, numel in ((2, 256 << 10), (2, 512 << 10), (2, 1 << 20), (2, 1_690_046), (2, 4_932_344), (8, 128 << 10),
                     (8, 256 << 10), (8, 512 << 10), (8, 1 << 20), (4, 3_900_000), (32, 256 << 10)):
        g = torch.Generator().manual_seed(n)
        ms = [nn.ParameterList([nn.Parameter(torch.randn(numel, generator=g))]) for _ in range(n)]
        w = [1.0 / n] * n
        reps = 50 if numel < (1 << 20) else 20
        r = {"n": n, "numel": numel, "input_MB": round(n * numel * 4 / 1e6, 2)}
        F._SMALL_ROW_BYTES = F._SMALL_ROUND_BYTES = 1 << 40
        r["small_us"] = med(lambda: F.FedAvg.aggregate(ms, w), reps)
        F._SMALL_ROUND_BYTES = 0
        r["native_us"] = med(lambda: F.FedAvg.aggregate(ms, w), reps)
        prev_min = F._NATIVE_MIN_CHUNK_BYTES
        F._NATIVE_MIN_CHUNK_BYTES = F._NATIVE_CHUNK_BYTES  # full 32 MiB chunks only
        r["native_32MiB_chunks_us"] = med(lambda: F.FedAvg.aggregate(ms, w), reps)
        F._NATIVE_MIN_CHUNK_BYTES = prev_min
        F.set_host_path("pipelined")
        r["pipelined_us"] = med(lambda: F.FedAvg.aggregate(ms, w), reps)
        F.set_host_path("native")
        F._SMALL_ROW_BYTES, F._SMALL_ROUND_BYTES = default
        r["default_us"] = med(lambda: F.FedAvg.aggregate(ms, w), reps)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
