"""Round 6: the result's parameter blocks taken on the walk extension's worker thread while the caller walks
the round's models (walk.cpp param_blocks_start / _finish; fedavg._ASYNC_BLOCKS) against taking them on the
caller's thread after the walk — FedAvg.aggregate end to end (synchronised), the two interleaved round by
round, medians of 100, the result kept until after the timing; every result compared bit for bit between
the two.  16 and 128 google_speech ResNet-34 bf16 models as one ParameterList each, 16 as the reference's
97-module tree.  It ran against commit bfbe4e3 (profiles/r06y, r06z); the worker thread was reverted after
r06z (the hand-off to it cost 100-200 us on that box), so fedavg._ASYNC_BLOCKS no longer exists."""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "decentralized-learning_amd"), os.path.join(ROOT, "tests")]
import bench  # noqa: E402


def main():
    from test_center_copy_layouts import tree_from_layout

    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    dev = torch.device("cuda", 0)
    cases = []
    for n in (16, 128):
        cases.append(("paramlist_%d" % n, bench._device_layout_models("google_speech_resnet34", n, torch.bfloat16, dev)[0]))
    trees = []
    for k in range(16):
        t = tree_from_layout("google_speech_resnet34").to(device=dev, dtype=torch.bfloat16)
        with torch.no_grad():
            for q in t.parameters():
                q.copy_(torch.randn(q.shape, generator=torch.Generator().manual_seed(k)) * 0.05)
        trees.append(t)
    cases.append(("tree_16", trees))
    for name, models in cases:
        n = len(models)
        w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
        ts = {True: [], False: []}
        res = {}
        for _ in range(3):
            for a in (True, False):
                fa._ASYNC_BLOCKS = a
                fa.FedAvg.aggregate(models, w)
        for _ in range(100):
            for a in (True, False):
                fa._ASYNC_BLOCKS = a
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = fa.FedAvg.aggregate(models, w)
                torch.cuda.synchronize()
                ts[a].append(time.perf_counter() - t0)
                res[a] = r
        fa._ASYNC_BLOCKS = True
        same = all(torch.equal(x.detach().view(torch.int16), y.detach().view(torch.int16))
                   for x, y in zip(res[True].parameters(), res[False].parameters()))
        print(json.dumps({"case": name, "async_us": round(statistics.median(ts[True]) * 1e6, 1),
                          "sync_us": round(statistics.median(ts[False]) * 1e6, 1), "same_bits": same}), flush=True)
        del res


if __name__ == "__main__":
    main()
