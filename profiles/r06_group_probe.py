"""Round 6: should device rounds of fewer than 64 models also be walked and launched in groups?  The
16-model ResNet-34 round starts its kernel ~104 us into the call, 42 us of it the layout walk of all 16
models (profiles/r06n); launching the first few models' fold after walking only them starts the GPU
earlier, at the price of one more pass over the result (dla_wsum_multi_table_acc).  FedAvg.aggregate end
to end (synchronised; the result kept until after the timing) with fedavg._GROUP_MIN / _DEVICE_GROUP_FIRST
set per variant, the variants interleaved round by round, medians of 60; every variant's result checked
bit for bit against the default's."""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "decentralized-learning_amd")]
import bench  # noqa: E402

VARIANTS = {"default": (64, 16), "group>=16,first4": (16, 4), "group>=16,first8": (16, 8)}
CONFIGS = [("google_speech_resnet34", 16, torch.bfloat16), ("google_speech_resnet34", 32, torch.bfloat16),
           ("cifar10_resnet8", 32, torch.float32), ("femnist_cnn", 32, torch.float32)]


def main():
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    dev = torch.device("cuda", 0)
    for name, n, dt in CONFIGS:
        try:
            models, p = bench._device_layout_models(name, n, dt, dev)
        except Exception as e:  # noqa: BLE001 — a layout this bench does not know
            print(json.dumps({"layout": name, "skipped": str(e)}), flush=True)
            continue
        w = [float(x) for x in np.random.default_rng(3).dirichlet(np.ones(n))]
        times = {v: [] for v in VARIANTS}
        outs = {}
        for _ in range(60):
            for v, (gmin, first) in VARIANTS.items():
                fa._GROUP_MIN, fa._DEVICE_GROUP_FIRST = gmin, first
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = fa.FedAvg.aggregate(models, w)
                torch.cuda.synchronize()
                times[v].append(time.perf_counter() - t0)
                outs[v] = res
        fa._GROUP_MIN, fa._DEVICE_GROUP_FIRST = VARIANTS["default"]
        ref = list(outs["default"].parameters())
        row = {"layout": name, "models": n, "dtype": str(dt), "params": p}
        for v in VARIANTS:
            same = all(torch.equal(a.detach().view(-1).view(torch.uint8), b.detach().view(-1).view(torch.uint8))
                       for a, b in zip(outs[v].parameters(), ref))
            row[v] = {"us": round(statistics.median(times[v]) * 1e6, 1), "same_bits": same}
        print(json.dumps(row), flush=True)
        del models, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
