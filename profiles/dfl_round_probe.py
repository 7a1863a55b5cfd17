"""r03: bench.py's dfl_round leg alone (8 EVA-block messages of a 25 M fp32 model -> DeviceModelManager
-> average -> serialize_model), with the per-peer ingress split into the wire split, the decode + gather
(loads_state_dict into the page-locked ingress buffer) and the stage call, on the process's NUMA node
as bench.py binds it.  Run it once per DLA_COPY_THREADS value to A/B the gather's threads.
Usage on the GPU box: DLA_COPY_THREADS=8 python profiles/dfl_round_probe.py"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402

from accdfl_amd.core import wire  # noqa: E402
from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402


def main():
    node = bind_to_gpu_node()
    dev = torch.device("cuda", 0)
    p, n = 25_000_000, 8
    msgs = bench.dfl_messages(n, p)
    row = bench.dfl_round(msgs, p, dev, reps=5)
    row["copy_threads"] = os.environ.get("DLA_COPY_THREADS", "8 (default)")
    row["numa_node_bound"] = node
    # per-peer split of the ingress: wrap the decode and the stage of DeviceModelManager
    phases = {"split": [], "decode_gather": [], "stage": []}
    orig_loads = wire.loads_state_dict

    def loads(*a, **kw):
        t0 = time.perf_counter()
        try:
            return orig_loads(*a, **kw)
        finally:
            phases["decode_gather"].append((time.perf_counter() - t0) * 1e3)
    wire.loads_state_dict = loads
    try:
        from accdfl_amd.core.peer_slab import PeerSlab
        st = PeerSlab.stage

        def stage(self, *a, **kw):
            t0 = time.perf_counter()
            try:
                return st(self, *a, **kw)
            finally:
                phases["stage"].append((time.perf_counter() - t0) * 1e3)
        PeerSlab.stage = stage
        for _ in range(3):
            t0 = time.perf_counter()
            for blocks, ml in msgs:
                ts = time.perf_counter()
                wire.split_blocks(blocks, ml)
                phases["split"].append((time.perf_counter() - ts) * 1e3)
            bench.dfl_round(msgs, p, dev, reps=1)
        PeerSlab.stage = st
    finally:
        wire.loads_state_dict = orig_loads
    row["per_peer_ms"] = {k: round(statistics.median(v), 3) for k, v in phases.items() if v}
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
