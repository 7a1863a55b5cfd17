"""Where FedAvg.aggregate's time goes outside dla_host_reduce for CPU modules of the BASELINE layouts
(_large_round: the one-pass layout walk, the result module's clone, the staging lookup, the native
call).  Usage on the GPU box: python profiles/host_phases_probe.py "configs[2],configs[3']"
Prints one JSON line per config: median ms of each phase over 5 calls after one warm call."""
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

print(json.dumps({"bound_to_numa_node": bind_to_gpu_node()}), flush=True)
cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["configs[2]", "configs[3']"]
for c in cfgs:
    name = [k for k in bench.HOST_CONFIGS if k.startswith(c + " ")][0]
    lay, n, dts = bench.HOST_CONFIGS[name]
    dt = torch.float32 if dts == "f32" else torch.bfloat16
    models, p = bench._layout_models(lay, n, dt, False)
    w = [1.0 / n] * n
    phases = {k: [] for k in ("layout", "fresh_params", "clone", "host_reduce_call", "aggregate_total",
                              "pre_native", "post_native")}
    stamps = {}
    orig = (fa._host_layout, fa._fresh_params, fa._clone_value, fa._lib.host_reduce_launch, fa._lib.HostReduceJob.join)

    depth = {}

    def timed(key, fn):
        def wrap(*a, **kw):  # the outermost call only (_clone_value recurses through the module name)
            depth[key] = depth.get(key, 0) + 1
            t0 = time.perf_counter()
            stamps.setdefault(key + "_enter", t0)
            try:
                return fn(*a, **kw)
            finally:
                depth[key] -= 1
                if depth[key] == 0:
                    t1 = time.perf_counter()
                    stamps[key + "_exit"] = t1
                    if key in phases:
                        phases[key].append((t1 - t0) * 1e3)
        return wrap

    fa._host_layout = timed("layout", orig[0])
    fa._fresh_params = timed("fresh_params", orig[1])
    fa._clone_value = timed("clone", orig[2])
    # the native round: from the (first) launch to the return of the (last) join
    fa._lib.host_reduce_launch = timed("launch", orig[3])
    fa._lib.HostReduceJob.join = timed("join", orig[4])
    try:
        for i in range(6):
            stamps.clear()
            t0 = time.perf_counter()
            fa.FedAvg.aggregate(models, w)
            t1 = time.perf_counter()
            phases["aggregate_total"].append((t1 - t0) * 1e3)
            if "launch_enter" in stamps:  # first launch in, last join out
                phases["pre_native"].append((stamps["launch_enter"] - t0) * 1e3)
                phases["post_native"].append((t1 - stamps["join_exit"]) * 1e3)
                phases["host_reduce_call"].append((stamps["join_exit"] - stamps["launch_enter"]) * 1e3)
    finally:
        (fa._host_layout, fa._fresh_params, fa._clone_value, fa._lib.host_reduce_launch,
         fa._lib.HostReduceJob.join) = orig
    row = {k: round(statistics.median(v[1:]), 3) for k, v in phases.items() if v}
    print(json.dumps(dict(config=c, peers=n, params=p, **row)), flush=True)
    del models
    fa.release_staging()
