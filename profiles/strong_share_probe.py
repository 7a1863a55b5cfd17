"""Rank 0's share of bench.py's strong-scaling lines at N = 1, 2, 4, 8, measured on ONE GPU (the
buckets every rank of an N-GPU run reduces are the same size): per-launch kernel time against the
ideal 1/N of the N = 1 time, with the same input rotation as the bench (HBM, not Infinity Cache).
Predicts the strong-scaling efficiency the driver's multi-GPU run will see for the reduce itself."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
bind_to_gpu_node(dev)
orig = bench.time_kernel
bench.time_kernel = lambda fn, steps, warmup, world, settle_s=None: orig(fn, steps, warmup, 1, settle_s)
base = {}
for n in (1, 2, 4, 8):
    rows = bench.strong_scaling(0, n, dev, 50, 5)
    for name, r in rows.items():
        us = r["kernel_us_max_rank"]
        base.setdefault(name, us)
        print(json.dumps({"model": name, "N": n, "bucket_params": r["bucket_params_max"], "kernel_us": us,
                          "ms_per_step": r["ms_per_step"], "ideal_us": round(base[name] / n, 2),
                          "reduce_efficiency": round(base[name] / n / us, 3), "kernel": r["kernel"]}), flush=True)
