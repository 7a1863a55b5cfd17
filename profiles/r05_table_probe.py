"""Round 5: where the non-kernel time of a device-module round's table reduce goes.

For the device_module_configs layouts, times the table reduce (dla_wsum_multi_table: the table's H2D
+ one wsum_multi_vec_kernel launch per 128-peer pass) back to back exactly as bench.py's reduce_us
does, under the table-upload mode the tuning build reads from DLA_TABLE_COPY (0: hipMemcpyAsync on
the stream, 1: a copy kernel on the stream, 2: a side-stream copy + event wait), and checks the result
bit for bit against the per-tensor path (dla_wsum_multi).  Run with ACCDFL_AMD_TUNING=1:

    ACCDFL_AMD_TUNING=1 DLA_TABLE_COPY=1 python profiles/r05_table_probe.py
"""
import ctypes
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

import bench  # noqa: E402
from accdfl_amd import _lib  # noqa: E402
from accdfl_amd.core import wsum  # noqa: E402
from accdfl_amd.core.gradient_aggregation import fedavg as fa  # noqa: E402

CONFIGS = {k: v for k, v in bench.DEVICE_CONFIGS.items() if sys.argv[1:] == [] or any(a in k for a in sys.argv[1:])}


def main():
    device = torch.device("cuda", 0)
    _lib.lib()
    mode = os.environ.get("DLA_TABLE_COPY", "0")
    for name, (lay, n, dts) in CONFIGS.items():
        dt = torch.float32 if dts == "f32" else torch.bfloat16
        es = 4 if dts == "f32" else 2
        models, p = bench._device_layout_models(lay, n, dt, device)
        w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
        byts = (n + 1) * p * es
        _, _, numels, table = fa._device_layout(models)
        center = fa._center_copy(models[0])
        outs = (ctypes.c_void_p * len(numels))(*[c.data_ptr() for c in center.parameters()])
        nums = (ctypes.c_int64 * len(numels))(*numels)
        ptrs = (ctypes.c_void_p * table.size).from_buffer(table)
        steps = 20 if byts > (256 << 20) else 100

        def reduce_once():
            wsum.wsum_multi_ptrs(dt, ptrs, outs, nums, w, device)

        evs = [bench.time_kernel(reduce_once, steps, 5, 1, settle_s=0.05)[1] for _ in range(5)]

        def e2e():
            fa.FedAvg.aggregate(models, w)
            torch.cuda.synchronize()

        e2e_ms = bench._median_ms(e2e, 20)

        def single():  # one table reduce on an idle GPU, until it is done (the latency a round sees)
            reduce_once()
            torch.cuda.synchronize()

        single_ms = bench._median_ms(single, 20)
        got = [c.detach().clone() for c in center.parameters()]
        old = wsum.MULTI_TABLE_MIN_PEERS, wsum.MULTI_TABLE_MIN_BYTES
        wsum.MULTI_TABLE_MIN_PEERS = wsum.MULTI_TABLE_MIN_BYTES = 1 << 62
        try:
            reduce_once()
        finally:
            wsum.MULTI_TABLE_MIN_PEERS, wsum.MULTI_TABLE_MIN_BYTES = old
        torch.cuda.synchronize()
        same = all(torch.equal(a.view(torch.int16 if es == 2 else torch.int32),
                               b.view(torch.int16 if es == 2 else torch.int32))
                   for a, b in zip(got, center.parameters()))
        us = [e / steps * 1e6 for e in evs]
        print(json.dumps({"config": name, "table_copy_mode": mode, "reduce_us_median": round(statistics.median(us), 2),
                          "reduce_us_all": [round(x, 2) for x in us],
                          "single_reduce_us": round(single_ms * 1e3, 1), "end_to_end_ms": round(e2e_ms, 4), "GB/s": round(byts / statistics.median(us) / 1e3, 1),
                          "table_bytes": _lib.wsum_multi_table_bytes(len(numels), n), "parity_vs_per_tensor": same}),
              flush=True)
        del models, center, got
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
