"""Round 5: the strong-scaling answer ("≥ 3.5x at 4 GPUs when bucket-sharded") predicted on one GPU.

For each fixed model of bench.py's STRONG lines, splits it into 2 / 4 / 8 parameter buckets exactly as
strong_line does (sharding.bucket_bounds, rotated input copies for buckets the Infinity Cache would
hold), times rank 0's bucket alone on this GPU with time_kernel, and divides the whole model's time on
the same GPU by it: the speedup an N-GPU node reaches if every GPU reduces its bucket as fast as this
one does and nothing else interferes (no barrier or collective costs included — the driver's SCALE run
measures those).  Prints one JSON line per model."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

import bench  # noqa: E402
from accdfl_amd.core.sharding import bucket_bounds  # noqa: E402


def share_s(n, m, dt, es, device, w, steps=40):
    pitch = max(128, (m + 127) // 128 * 128)
    set_bytes = (n + 1) * pitch * es
    copies = 1 if set_bytes >= bench._ROTATE_BYTES else min(64, -(-bench._ROTATE_BYTES // set_bytes))
    inputs = [bench.SlabInput(n, m, dt, device, 1000 + 131 * c, w) for c in range(copies)]
    sp = torch.cuda.current_stream().cuda_stream
    ctr = [0]

    def step():
        inputs[ctr[0] % len(inputs)].launch(sp)
        ctr[0] += 1
    wall, ev = bench.time_kernel(step, steps, 5, 1)
    del inputs
    torch.cuda.empty_cache()
    return wall / steps, ev / steps, copies


def main():
    device = torch.device("cuda", 0)
    for name, (n, params, dts) in bench.STRONG.items():
        dt = torch.float32 if dts == "f32" else torch.bfloat16
        es = 4 if dts == "f32" else 2
        w = [float(x) for x in np.random.default_rng(0).dirichlet(np.ones(n))]
        whole, whole_ev, _ = share_s(n, params, dt, es, device, w)
        row = {"model": name, "peers": n, "params": params, "one_gpu_us": round(whole * 1e6, 2)}
        for world in (2, 4, 8):
            s, e = bucket_bounds(params, world, 256 // es)[0]
            t, t_ev, copies = share_s(n, e - s, dt, es, device, w)
            row["n%d" % world] = {"bucket_params": e - s, "us_per_step": round(t * 1e6, 2),
                                  "kernel_us": round(t_ev * 1e6, 2), "rotated_copies": copies,
                                  "predicted_speedup": round(whole / t, 3),
                                  "predicted_efficiency": round(whole / t / world, 3)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
