"""Host-inclusive FedAvg.aggregate on CPU modules of the BASELINE layouts, per host path and
staging setting (A/B for dla_host_reduce).  Usage on the GPU box:
    DLA_HOST_REDUCE_STATS=1 DLA_COPY_THREADS=16 ACCDFL_AMD_HOST_CHUNK_MB=32 python profiles/host_reduce_probe.py
Prints one JSON line per config: median ms of 3 calls after one warm call."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402

from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg, host_path, release_staging  # noqa: E402

if os.environ.get("PROBE_BIND") == "gpu":
    from accdfl_amd.core.host_memory import bind_to_gpu_node
    print(json.dumps({"bound_to_numa_node": bind_to_gpu_node()}), flush=True)
cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["ns", "configs[3']", "configs[4]"]
env = {k: os.environ.get(k) for k in ("DLA_COPY_THREADS", "ACCDFL_AMD_HOST_CHUNK_MB", "ACCDFL_AMD_HOST_PATH",
                                      "PROBE_BIND")}
for c in cfgs:
    if c == "ns":
        row = bench.host_inclusive(8, 25_000_000)
        print(json.dumps(dict(config=c, env=env, path=host_path(), ms=row["ms"], GBps=row["value"])), flush=True)
        continue
    name = [k for k in bench.HOST_CONFIGS if k.startswith(c + " ")][0]
    lay, n, dts = bench.HOST_CONFIGS[name]
    dt = torch.float32 if dts == "f32" else torch.bfloat16
    for mem in ("pageable", "pinned"):
        models, p = bench._layout_models(lay, n, dt, mem == "pinned")
        w = [1.0 / n] * n
        ms = bench._median_ms(lambda: FedAvg.aggregate(models, w), 3)
        es = 4 if dts == "f32" else 2
        print(json.dumps(dict(config=c, mem=mem, env=env, path=host_path(), ms=ms,
                              GBps=round((n + 1) * p * es / ms / 1e6, 2))), flush=True)
        del models
    release_staging()
