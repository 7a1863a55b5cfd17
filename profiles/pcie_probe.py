"""PCIe ceilings of this box for the host path: H2D of page-locked memory as one copy, split over
2 or 4 streams (several DMA engines), the D2H direction, both directions at once, and a kernel
reading page-locked host memory directly (zero-copy, what dla_host_round_start does).  Usage on the
GPU box: python profiles/pcie_probe.py [MB]  -> one JSON line per measurement (GB/s, median of 5)."""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402

print(json.dumps({"bound_to_numa_node": bind_to_gpu_node()}), flush=True)
mb = int(sys.argv[1]) if len(sys.argv) > 1 else 256
nbytes = mb << 20
h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).fill_(1)
h2 = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
d2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
streams = [torch.cuda.Stream() for _ in range(4)]


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def split_copy(dst, src, parts):
    step = nbytes // parts
    for i in range(parts):
        with torch.cuda.stream(streams[i]):
            dst[i * step:(i + 1) * step].copy_(src[i * step:(i + 1) * step], non_blocking=True)


for parts in (1, 2, 4):
    t = timed(lambda: split_copy(d, h, parts))
    print(json.dumps({"h2d_streams": parts, "MB": mb, "GB/s": round(nbytes / t / 1e9, 2)}), flush=True)
for parts in (1, 2):
    t = timed(lambda: split_copy(h2, d, parts))
    print(json.dumps({"d2h_streams": parts, "MB": mb, "GB/s": round(nbytes / t / 1e9, 2)}), flush=True)


def both():
    with torch.cuda.stream(streams[0]):
        d.copy_(h, non_blocking=True)
    with torch.cuda.stream(streams[1]):
        h2.copy_(d2, non_blocking=True)


t = timed(both)
print(json.dumps({"h2d_and_d2h_at_once": True, "MB_each": mb, "GB/s_each": round(nbytes / t / 1e9, 2)}), flush=True)
# zero-copy: the reduce kernel reading page-locked host memory across PCIe (dla_host_round_start's
# access pattern): one and four "peers" in host memory, output in HBM
from accdfl_amd import _lib  # noqa: E402

sp = torch.cuda.current_stream().cuda_stream
out = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda")
for peers in (1, 4):
    per = nbytes // 4 // peers
    ptrs = [h.data_ptr() + k * per * 4 for k in range(peers)]
    t = timed(lambda: _lib.wsum_ptrs(_lib.DLA_F32, ptrs, [1.0 / peers] * peers, per, out.data_ptr(), sp))
    print(json.dumps({"zero_copy_kernel_read_peers": peers, "MB": mb, "GB/s": round(nbytes / t / 1e9, 2)}),
          flush=True)
for chunk_mb in (4, 16, 64):
    step = chunk_mb << 20
    t = timed(lambda: [d[i:i + step].copy_(h[i:i + step], non_blocking=True) for i in range(0, nbytes, step)])
    print(json.dumps({"h2d_chunked_MB": chunk_mb, "GB/s": round(nbytes / t / 1e9, 2)}), flush=True)
