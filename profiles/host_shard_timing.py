"""Host-inclusive FedAvg.aggregate on CPU modules, bucket-sharded over G device slots, with
one host thread per slot vs the serial peer-major issue (diagnostic, GPU box).

Usage: python profiles/host_shard_timing.py [G] [devices]   devices: "same" puts every slot
on cuda:0 (a 1-GPU box: all buckets share one PCIe link, so only the host-side packing
parallelism shows), "distinct" uses cuda:0..G-1."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
import torch  # noqa: E402
from torch import nn  # noqa: E402

from accdfl_amd.core.gradient_aggregation import fedavg as fa  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 3
mode = sys.argv[2] if len(sys.argv) > 2 else "same"
n, p = 8, 25_000_000
gen = torch.Generator().manual_seed(2000)
models = []
for _ in range(n):
    m = nn.Module()
    m.w = nn.Parameter(torch.randn(p, generator=gen) * 0.05)
    models.append(m)
w = [1.0 / n] * n
res = {}
for g, threads in ((1, False), (1, True), (G, False), (G, True)):
    fa.set_host_devices([0] * g if mode == "same" else list(range(g)))
    fa.set_shard_threads(threads)
    fa.FedAvg.aggregate(models, w)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        fa.FedAvg.aggregate(models, w)
        ts.append(time.perf_counter() - t0)
    fa.release_staging()
    fa.set_shard_threads(True)
    res["%d_%s" % (g, "pipelined" if threads else "packed")] = round(statistics.median(ts) * 1e3, 2)
print(json.dumps({"slots": G, "devices": mode, "ms": res, "torch_threads": torch.get_num_threads()}))
