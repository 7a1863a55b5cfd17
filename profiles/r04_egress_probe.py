"""r04: egress of an averaged 25 M fp32 row from HBM into serialize_model bytes (wire.dumps_state_dict over a
DeviceSource: chunked D2H through two page-locked bounce buffers, each chunk copied out by the threaded
memcpy while the next one's D2H runs) at the chunk size ACCDFL_AMD_EGRESS_CHUNK_MB of this process (r04y: and the chunk ramp
ACCDFL_AMD_EGRESS_RAMP of that tree, since removed),
bound to the GPU's NUMA node (EGRESS_NO_BIND=1: not bound).
Prints one JSON line: the median ms of 15 encodes and the bytes' check against the row.
Usage on the GPU box: ACCDFL_AMD_EGRESS_CHUNK_MB=8 python profiles/r04_egress_probe.py"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

import torch  # noqa: E402

from accdfl_amd.core import wire  # noqa: E402
from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402


def main():
    node = bind_to_gpu_node() if os.environ.get("EGRESS_NO_BIND") != "1" else None
    flat = torch.randn(25_000_000, generator=torch.Generator().manual_seed(5)).cuda()
    src = wire.DeviceSource(flat, 0, (25_000_000,))
    ts, frees = [], []
    data = None
    for _ in range(16):
        tf = time.perf_counter()
        del data  # the previous payload's unmap, timed apart (not part of the encode)
        frees.append(time.perf_counter() - tf)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        data = wire.dumps_state_dict({"w": src})
        ts.append(time.perf_counter() - t0)
    ok = data == wire.dumps_state_dict({"w": flat.cpu()})
    print(json.dumps({"numa_node_bound": node, "chunk_MB": wire._EGRESS_CHUNK >> 20, "ramp": getattr(wire, "_EGRESS_RAMP", None), "egress_ms": round(statistics.median(ts[1:]) * 1e3, 3),
                      "min_ms": round(min(ts[1:]) * 1e3, 3), "free_ms": round(statistics.median(frees[2:]) * 1e3, 3),
                      "bytes_equal": ok}), flush=True)


if __name__ == "__main__":
    main()
