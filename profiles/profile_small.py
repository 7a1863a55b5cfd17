"""Where does FedAvg.aggregate spend its time on small CPU models? (diagnostic, GPU box)"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # repo root
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
import torch  # noqa: E402
from torch import nn  # noqa: E402

from accdfl_amd.core.gradient_aggregation import fedavg as fa  # noqa: E402

shapes = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,), (64, 32, 5, 5), (64,), (64,),
          (64,), (10, 576), (10,)]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
models = [nn.ParameterList([nn.Parameter(torch.randn(s) * 0.05) for s in shapes]) for _ in range(n)]
w = [1.0 / n] * n
for _ in range(20):
    fa.FedAvg.aggregate(models, w)
t0 = time.perf_counter()
for _ in range(200):
    fa.FedAvg.aggregate(models, w)
print("aggregate ms", (time.perf_counter() - t0) / 200 * 1e3)
t0 = time.perf_counter()
for _ in range(200):
    fa._center_copy(models[0])
print("center_copy ms", (time.perf_counter() - t0) / 200 * 1e3)
pr = cProfile.Profile()
pr.enable()
for _ in range(200):
    fa.FedAvg.aggregate(models, w)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
