"""Round 6: does the device-module table reduce run faster in passes over fewer peers?
The kernel is bound by address translation (each wave reads one page of every peer's tensor; UTCL2 busy
60 % at 16 models, 98 % at 128, against 1-5 % for a slab of the same bytes: profiles/r05h).  Passes over
fewer peers keep fewer pages in flight per wave, at the cost of one more read + write of the result per
pass (dla_wsum_multi_table_acc continues the fold in the result: the same bits).  For each config the
same walked layout is reduced with the peers split into passes of the given sizes, back to back, HIP
events over 20 rounds, the variants interleaved over 3 rounds; every variant's result is compared with
the one-pass result bit for bit."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "decentralized-learning_amd")]
import bench  # noqa: E402

CONFIGS = [
    ("google_speech_resnet34", 16, torch.bfloat16, [[16], [8, 8]]),
    ("google_speech_resnet34", 128, torch.bfloat16, [[128], [64, 64], [32, 32, 32, 32], [16, 48, 64]]),
    ("cifar10_resnet8", 64, torch.float32, [[64], [32, 32], [16, 48]]),
]


def main():
    from accdfl_amd.core import wsum as _wsum
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    dev = torch.device("cuda", 0)
    for name, n, dt, variants in CONFIGS:
        models, p = bench._device_layout_models(name, n, dt, dev)
        dtype, device, numels, table = fa._device_layout(models)
        w = [float(x) for x in np.random.default_rng(7).dirichlet(np.ones(n))]
        nums = fa._flat_plan(dtype, numels)[3]
        total = sum(numels)
        plans = {}
        for v in variants:
            passes, a = [], 0
            for k in v:
                sub = np.ascontiguousarray(table[:, a:a + k])
                passes.append(((ctypes.c_void_p * sub.size).from_buffer(sub), w[a:a + k], a > 0, sub))
                a += k
            assert a == n
            outs_t = [torch.empty(k, dtype=dtype, device=dev) for k in numels]
            outs = (ctypes.c_void_p * len(numels))(*[o.data_ptr() for o in outs_t])
            plans[tuple(v)] = (passes, outs, outs_t)

        def run(v):
            passes, outs, _ = plans[v]
            for ptrs, ww, acc, _sub in passes:
                _wsum.wsum_multi_ptrs(dtype, ptrs, outs, nums, ww, device, acc_in=acc, total_elems=total)

        times = {v: [] for v in plans}
        for _ in range(3):
            for v in plans:
                for _ in range(5):
                    run(v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    run(v)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(round(e0.elapsed_time(e1) * 1e3 / 20, 1))
        ref = plans[tuple(variants[0])][2]
        es = ref[0].element_size()
        algo = (n + 1) * total * es
        for v in plans:
            same = all(torch.equal(a.view(torch.uint8), b.view(torch.uint8)) for a, b in zip(plans[v][2], ref))
            print(json.dumps({"layout": name, "models": n, "dtype": str(dt), "passes": list(v), "us": times[v],
                              "one_pass_GBps_equiv": round(algo / (min(times[v]) / 1e6) / 1e9, 1),
                              "same_bits_as_one_pass": same}), flush=True)
        del models, plans
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
