"""r04: how a peer's row can land in the tile-interleaved PeerSlab without the contiguous device row and
the on-device scatter, and how page-locked peers can skip the pack (next 4).

Measured, each the median of 5 (GB/s of the peer's bytes):
  * a 100 MB H2D from page-locked memory as one contiguous copy (the link rate, the reference point);
  * the same bytes as ONE hipMemcpy2DAsync into row k of a [n_tiles, rows, tile] slab (width = tile
    bytes, destination pitch = rows x tile bytes) for 4 / 16 / 32 KiB tiles, from page-locked and from
    pageable (already touched) memory;
  * the round-3 path: contiguous H2D into a device row, then the torch strided copy into the tiles;
  * a device row -> tiles as one 2D D2D copy against the torch strided copy;
  * zero-copy: the reduce kernel reading N page-locked peers across PCIe (dla_wsum on host pointers,
    which torch's page-locked memory maps at the same address) for the configs[2] and north-star
    shapes, against the DMA rate.
Usage on the GPU box: python profiles/r04_copy_probe.py  -> one JSON line per measurement."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

from accdfl_amd import _lib  # noqa: E402
from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402

print(json.dumps({"bound_to_numa_node": bind_to_gpu_node()}), flush=True)
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                 ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpy2DAsync.restype = ctypes.c_int
H2D, D2D = 1, 3
stream = torch.cuda.current_stream()
sp = stream.cuda_stream


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


def emit(**kw):
    print(json.dumps(kw), flush=True)


nbytes = 100_000_000
pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).fill_(3)
pageable = torch.empty(nbytes, dtype=torch.uint8).fill_(5)
row = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
t = timed(lambda: row.copy_(pinned, non_blocking=True))
emit(what="h2d_contiguous_pinned", GBps=round(nbytes / t / 1e9, 2))
t = timed(lambda: row.copy_(pageable, non_blocking=True))
emit(what="h2d_contiguous_pageable", GBps=round(nbytes / t / 1e9, 2))


def copy2d(dst_base, k, tile, rows, src, n, kind):
    full = n // tile
    if full:
        rc = hip.hipMemcpy2DAsync(dst_base + k * tile, rows * tile, src, tile, tile, full, kind, sp)
        assert rc == 0, rc
    rest = n - full * tile
    if rest:
        rc = hip.hipMemcpy2DAsync(dst_base + (full * rows + k) * tile, rest, src + full * tile, rest, rest, 1, kind, sp)
        assert rc == 0, rc


for tile_kib, rows in ((4, 128), (16, 16), (32, 8)):
    tile = tile_kib << 10
    n_tiles = -(-nbytes // tile)
    slab = torch.empty((n_tiles, rows, tile), dtype=torch.uint8, device="cuda")
    k = rows // 2
    for src_name, src in (("pinned", pinned), ("pageable", pageable)):
        t = timed(lambda: copy2d(slab.data_ptr(), k, tile, rows, src.data_ptr(), nbytes, H2D))
        # check: row k's tiles hold the source
        ok = bool(torch.equal(slab[:, k, :].reshape(-1)[:nbytes].cpu(), src))
        emit(what="h2d_2d_into_tiles", src=src_name, tile_KiB=tile_kib, rows=rows, GBps=round(nbytes / t / 1e9, 2),
             ok=ok)
    full = nbytes // tile

    def scatter():
        row.copy_(pinned, non_blocking=True)
        slab[:full, k, :].copy_(row[: full * tile].view(full, tile))
        slab[full, k, : nbytes - full * tile].copy_(row[full * tile:])
    t = timed(scatter)
    emit(what="h2d_then_torch_scatter", tile_KiB=tile_kib, rows=rows, GBps=round(nbytes / t / 1e9, 2))
    t = timed(lambda: copy2d(slab.data_ptr(), k, tile, rows, row.data_ptr(), nbytes, D2D))
    emit(what="d2d_2d_into_tiles", tile_KiB=tile_kib, rows=rows, GBps=round(nbytes / t / 1e9, 2),
         us=round(t * 1e6, 1))

    def tscatter():
        slab[:full, k, :].copy_(row[: full * tile].view(full, tile))
        slab[full, k, : nbytes - full * tile].copy_(row[full * tile:])
    t = timed(tscatter)
    emit(what="d2d_torch_scatter", tile_KiB=tile_kib, rows=rows, GBps=round(nbytes / t / 1e9, 2), us=round(t * 1e6, 1))
    del slab
    torch.cuda.empty_cache()

# zero-copy reduce of page-locked peers (the pinned-peer host path without a pack or a DMA)
del row
for name, n, p, dt, code, es in (("configs2_femnist", 32, 1_690_046, torch.float32, _lib.DLA_F32, 4),
                                 ("north_star", 8, 25_000_000, torch.float32, _lib.DLA_F32, 4),
                                 ("configs4_share", 128, 2_662_045, torch.bfloat16, _lib.DLA_BF16, 2)):
    peers = [torch.empty(p, dtype=dt, pin_memory=True).fill_(0.5 + k) for k in range(n)]
    out = torch.empty(p, dtype=dt, device="cuda")
    w = [1.0 / n] * n
    ptrs = [x.data_ptr() for x in peers]
    t = timed(lambda: _lib.wsum_ptrs(code, ptrs, w, p, out.data_ptr(), sp))
    dev = torch.empty((n, p), dtype=dt, device="cuda")
    t2 = timed(lambda: [dev[k].copy_(peers[k], non_blocking=True) for k in range(n)])
    emit(what="zero_copy_reduce_pinned_peers", shape=name, peers=n, params=p, ms=round(t * 1e3, 3),
         GBps=round(n * p * es / t / 1e9, 2), dma_per_peer_ms=round(t2 * 1e3, 3),
         dma_GBps=round(n * p * es / t2 / 1e9, 2), kernel=_lib.select_kernel(code, n, p))
    del peers, out, dev
    torch.cuda.empty_cache()
