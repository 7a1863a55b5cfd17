"""r04: the small-round / pipelined-round crossover for CPU models (fedavg._is_small) re-measured on the
round-4 host paths (both now read page-locked rows with the kernel across PCIe).  For CPU modules of the
reference layouts (pageable), FedAvg.aggregate with the small-round path allowed (the default bounds) and
forced off (fa._SMALL_ROUND_BYTES = 0: the pipelined dla_host_reduce path), interleaved, results checked
bit-exact against each other.  Prints one JSON line per (layout, peers): median ms of each.
Usage on the GPU box: python profiles/r04_small_large_ab.py"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402

from accdfl_amd.core.gradient_aggregation import fedavg as fa  # noqa: E402
from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402


def med_ms(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


def main():
    print(json.dumps({"numa_node_bound": bind_to_gpu_node()}), flush=True)
    default = fa._SMALL_ROUND_BYTES
    for lay, n in (("gnlenet", 8), ("gnlenet", 64), ("femnist_cnn", 2), ("femnist_cnn", 4), ("femnist_cnn", 8),
                   ("cifar10_resnet8", 2), ("cifar10_resnet8", 4)):
        models, p = bench._layout_models(lay, n, torch.float32, False)
        w = [1.0 / n] * n
        res = {"small": [], "pipelined": []}
        outs = {}
        for _ in range(4):
            for name, bound in (("small", default), ("pipelined", 0)):
                fa._SMALL_ROUND_BYTES = bound
                outs[name] = torch.cat([q.detach().reshape(-1) for q in fa.FedAvg.aggregate(models, w).parameters()])
                res[name].append(med_ms(lambda: fa.FedAvg.aggregate(models, w), 10))
        fa._SMALL_ROUND_BYTES = default
        same = torch.equal(outs["small"].view(torch.int32), outs["pipelined"].view(torch.int32))
        print(json.dumps({"layout": lay, "peers": n, "MB": round(n * p * 4 / 1e6, 1), "bit_exact": same,
                          **{k: round(statistics.median(v), 3) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
