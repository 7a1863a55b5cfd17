"""r04: FedAvg.aggregate on CPU modules (pageable, the reference's call sites) of small rounds — the GL merge
of two models and small DFL / DL rounds — which take the small-round path (dla_host_round_start: one
pack into page-locked rows, the kernel reading them and writing the page-locked result across PCIe).
Median ms of 30 calls per (layout, peers), process bound to the GPU's NUMA node.  Run once per library
setting (product; tuning build with DLA_HOST_AUTO_KERNEL=1 for the shape-chosen kernel) -> JSON lines."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402

from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg  # noqa: E402
from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402

bind_to_gpu_node()
out = {"tuning": os.environ.get("ACCDFL_AMD_TUNING", "") == "1",
       "auto_kernel": os.environ.get("DLA_HOST_AUTO_KERNEL") is not None}
for lay, n in (("gnlenet", 2), ("gnlenet", 8), ("femnist_cnn", 2), ("femnist_cnn", 8), ("cifar10_resnet8", 2),
               ("cifar10_resnet8", 4)):
    models, p = bench._layout_models(lay, n, torch.float32, False)
    w = [1.0 / n] * n
    FedAvg.aggregate(models, w)
    ts = []
    for _ in range(30):
        t0 = time.perf_counter()
        FedAvg.aggregate(models, w)
        ts.append(time.perf_counter() - t0)
    out["%s x %d" % (lay, n)] = round(statistics.median(ts) * 1e3, 3)
print(json.dumps(out), flush=True)
