"""Round 6: does the table kernel's address-translation load come from the device
modules' allocation granularity?  16 and 128 google_speech ResNet-34 bf16 device models reduced by
wsum_multi_ptrs (dla_wsum_multi_table, wsum_multi_vec_kernel) in two layouts of the SAME parameters:
  separate   — one caching-allocator block per parameter (what .to(device) / clone leaves: bench.py
               _device_layout_models, today's device_module_configs);
  contiguous — each model's parameters as 256-byte aligned views of ONE allocation per model;
beside the tile-interleaved flat slab of the same bytes.  HIP events over back-to-back launches (bench.py
time_kernel), medians of 3; one JSON line per (models, layout).  The counters of the same launches come
from profiles/pmc_driver.py r34x16,r34x16c,r34x128,r34x128c (profiles/r06c_run.sh)."""
import ctypes
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "decentralized-learning_amd"), os.path.join(ROOT, "profiles")]
import bench  # noqa: E402
from pmc_driver import contiguous_model  # noqa: E402


def main():
    from accdfl_amd.core import wsum

    dev = torch.device("cuda", 0)
    shapes, _ = bench._layout("google_speech_resnet34")
    numels = [int(np.prod(s)) if s else 1 for s in shapes]
    p = sum(numels)
    for n in (16, 128):
        w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
        byts = (n + 1) * p * 2
        steps = 20 if n > 16 else 100
        row = {"models": n, "tensors_per_model": len(numels), "bytes": byts}
        # separate twice: drift between the runs; "staggered": contiguous, model k shifted by k x 4.25 KiB
        # (do same-offset reads of the models landing on the same channels explain "contiguous"?)
        for layout in ("separate", "contiguous", "staggered", "separate_again"):
            if layout == "contiguous":
                peers = [contiguous_model(numels, torch.bfloat16, dev) for _ in range(n)]
            elif layout == "staggered":
                peers = [contiguous_model(numels, torch.bfloat16, dev, shift_bytes=k * 4352) for k in range(n)]
            else:
                peers = [[torch.empty(m, dtype=torch.bfloat16, device=dev) for m in numels] for _ in range(n)]
            for ts in peers:
                for t in ts:
                    t.normal_(0, 0.05)
            outs = [torch.empty(m, dtype=torch.bfloat16, device=dev) for m in numels]
            ptrs = (ctypes.c_void_p * (n * len(numels)))(*[peers[k][t].data_ptr() for t in range(len(numels))
                                                           for k in range(n)])
            out_p = (ctypes.c_void_p * len(numels))(*[o.data_ptr() for o in outs])
            nums = (ctypes.c_int64 * len(numels))(*numels)

            def once():
                wsum.wsum_multi_ptrs(torch.bfloat16, ptrs, out_p, nums, w, dev)

            ev = statistics.median(bench.time_kernel(once, steps, 5, 1, settle_s=0.05)[1] for _ in range(3))
            us = ev / steps * 1e6
            key = layout
            row[key + "_us"] = round(us, 2)
            row[key + "_frac_of_8TBps"] = round(byts / (us * 1e-6) / 8e12, 4)
            del peers, outs
            torch.cuda.empty_cache()
        inp = bench.SlabInput(n, p, torch.bfloat16, dev, 1000, w)
        sp = torch.cuda.current_stream().cuda_stream
        ev = statistics.median(bench.time_kernel(lambda: inp.launch(sp), steps, 5, 1, settle_s=0.05)[1]
                               for _ in range(3))
        row["flat_slab_us"] = round(ev / steps * 1e6, 2)
        del inp
        torch.cuda.empty_cache()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
