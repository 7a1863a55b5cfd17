import os, sys, time, statistics, torch
sys.path.insert(0, "/root/repo/decentralized-learning_amd")
from torch import nn
from accdfl_amd.core.gradient_aggregation import fedavg as F
from accdfl_amd.core.host_memory import bind_to_gpu_node
bind_to_gpu_node()
for n, numel in ((2, 4_932_344), (8, 1 << 20)):
    g = torch.Generator().manual_seed(n)
    ms = [nn.ParameterList([nn.Parameter(torch.randn(numel, generator=g))]) for _ in range(n)]
    w = [1.0 / n] * n
    F._SMALL_ROUND_BYTES = 0
    for _ in range(3): F.FedAvg.aggregate(ms, w)
    print("== native", n, numel, flush=True)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter(); F.FedAvg.aggregate(ms, w); ts.append(time.perf_counter() - t0)
    print("native ms", [round(t * 1e3, 3) for t in ts], flush=True)
    t0 = time.perf_counter(); c = F._center_copy(ms[0], large=False); print("center_copy ms", (time.perf_counter() - t0) * 1e3)
    t0 = time.perf_counter(); c.__dict__  # noqa
    buf = torch.empty(numel); t0 = time.perf_counter(); buf.fill_(1.0); print("fresh fill ms", (time.perf_counter() - t0) * 1e3, flush=True)
