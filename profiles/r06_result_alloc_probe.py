"""Round 6: what allocator-visible device results cost.  For a google_speech ResNet-34
bf16 device model (110 parameters, 108 BN buffers), the host time of each way to make the result's tensors:
  param_fresh    — walk.cpp param_fresh: one caching-allocator block per parameter (round 6);
  param_views    — the round-4/5 layout: one torch.empty for all parameters + walk.cpp param_views aliases;
  buffer_copies  — walk.cpp buffer_copies (round 6: a block per buffer, one fused copy);
  tensors        — walk.cpp tensors (models[0]'s parameter and buffer lists);
medians of 200 calls (results dropped between calls, so the allocator serves them from its cache); then
FedAvg.aggregate end to end on 16 and 128 such models (synchronised), medians of 20."""
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


def med(fn, reps=200):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def main():
    from accdfl_amd import _lib
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    dev = torch.device("cuda", 0)
    mod = _lib.walk_module()
    models, p = bench._device_layout_models("google_speech_resnet34", 128, torch.bfloat16, dev)
    fa._plain_walk(type(models[0]))
    for sub in models[0].modules():
        fa._plain_walk(type(sub))
    p0, b0 = mod.tensors(models[0], fa._PLAIN_SET)
    numels = [x.numel() for x in p0]
    offs, total, _, _ = fa._flat_plan(torch.bfloat16, numels)
    out = {"parameters": len(p0), "buffers": len(b0)}
    out["tensors_us"] = med(lambda: mod.tensors(models[0], fa._PLAIN_SET))
    out["param_fresh_us"] = med(lambda: mod.param_fresh(p0, {}))

    def views():
        flat = torch.empty(total, dtype=torch.bfloat16, device=dev)
        mod.param_views(flat, p0, offs, {})
    out["param_views_us"] = med(views)
    out["buffer_copies_us"] = med(lambda: mod.buffer_copies(b0, {}))
    # its two halves: one allocator block per buffer (param_fresh makes the same blocks, as Parameters), and
    # the fused copy into blocks made beforehand
    out["buffer_blocks_only_us"] = med(lambda: mod.param_fresh(b0, {}))
    dsts = [torch.empty_like(b) for b in b0]
    out["foreach_copy_only_us"] = med(lambda: torch._foreach_copy_(dsts, b0))
    torch.cuda.synchronize()
    w = [float(x) for x in np.random.default_rng(1).dirichlet(np.ones(128))]
    for n in (16, 128):
        ww = [x / sum(w[:n]) for x in w[:n]]

        def e2e():
            fa.FedAvg.aggregate(models[:n], ww)
            torch.cuda.synchronize()
        e2e()
        out["aggregate_%d_models_ms" % n] = round(med(e2e, 20) / 1e3, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
