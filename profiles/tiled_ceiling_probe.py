"""r02: the north star's access pattern without its arithmetic, as a ceiling for the product
kernel.  8 peers x 100 MB in the tile-interleaved layout ([tiles][8][T], T = 1, 4 or 16 KiB),
one 16-byte vector per lane per peer XOR-folded and written (probe dlp_tiled8, sc1 store), the
write either to a separate flat buffer or into a 9th slot of each tile group; beside it the
8-stream read alone over the same bytes as one flat buffer (dlp_read) and the 100 MB sc1 write
alone (dlp_write), and the product kernel (dla_wsum_slab_tiled, 16 KiB tiles)."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
from accdfl_amd import _lib  # noqa: E402


def ev_time(fn, reps=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    so = ctypes.CDLL(_lib.build_probe())
    vp = ctypes.c_void_p
    so.dlp_tiled8.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int, ctypes.c_int, vp]
    so.dlp_read.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int, ctypes.c_int, vp]
    so.dlp_write.argtypes = [vp, ctypes.c_int64, ctypes.c_int, vp]
    n, p = 8, 25_000_000
    each = p * 4
    slab = torch.empty(9 * each // 4 + 65536, dtype=torch.float32, device="cuda").normal_()
    out = torch.empty(p + 4096, dtype=torch.float32, device="cuda")
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    sp = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    te = 16384 // 4
    w = [1.0 / n] * n
    legs = {
        "read_800MB_flat": lambda: so.dlp_read(slab.data_ptr(), 8 * each, sink.data_ptr(), 4, 1, sp()),
        "write_100MB_sc1": lambda: so.dlp_write(out.data_ptr(), each, 1, sp()),
        "product_tiled16K": lambda: _lib.wsum_slab_tiled_ptr(0, slab.data_ptr(), te, n, w, p, out.data_ptr(), sp()),
    }
    for ch in (1, 4, 16):
        for slot in (0, 1):
            legs["xor_tiled_%dKiB_outslot%d" % (ch, slot)] = (
                lambda ch=ch, slot=slot: so.dlp_tiled8(slab.data_ptr(), each, out.data_ptr(), ch, slot, sp()))
    res = {k: [] for k in legs}
    for _ in range(5):
        for k, fn in legs.items():
            res[k].append(ev_time(fn))
    for k in legs:
        t = statistics.median(res[k])
        byts = 8 * each if k.startswith("read") else each if k.startswith("write") else 9 * each
        print(json.dumps({"leg": k, "us": round(t, 2), "GB/s": round(byts / t / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
