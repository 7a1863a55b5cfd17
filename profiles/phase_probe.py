"""Is the north-star reduce's gap to the pure-read ceiling the read/write mix itself?
Times, at the north-star size (8 x 100 MB in, 100 MB out, beyond the 256 MB MALL):
  read8      8-stream read, no write (probe dlp_mread8 write=0)
  write      100 MB write stream alone (probe dlp_write, plain and sc1)
  read8+w    the FedAvg access pattern, sc1 write (dlp_mread8 write=2)
  wsum       the product kernel
If read8 + write (run one after the other) is well below read8+w, separating the reads from
the writes in time (phases) could pay; if not, the mix costs nothing extra."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
from accdfl_amd import _lib  # noqa: E402


def ev_time(fn, reps=30, warm=3):
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
    so.dlp_write.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    so.dlp_mread8.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_int, ctypes.c_void_p]
    n, p = 8, 25_000_000
    slab = torch.empty((n, p + 64), dtype=torch.float32, device="cuda").normal_()
    out = torch.empty(p, dtype=torch.float32, device="cuda")
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    each = p * 4
    arr = (ctypes.c_void_p * 8)(*[slab[k].data_ptr() for k in range(n)])
    sp = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    ptrs = [slab[k].data_ptr() for k in range(n)]
    w = [1.0 / n] * n
    so.dlp_bigtile8.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                ctypes.c_int, ctypes.c_void_p]
    wf = (ctypes.c_float * 8)(*w)
    legs = {
        "read8": lambda: so.dlp_mread8(arr, each, out.data_ptr(), sink.data_ptr(), 1, 0, sp()),
        "write_plain": lambda: so.dlp_write(out.data_ptr(), each, 0, sp()),
        "write_sc1": lambda: so.dlp_write(out.data_ptr(), each, 1, sp()),
        "read8+w_sc1": lambda: so.dlp_mread8(arr, each, out.data_ptr(), sink.data_ptr(), 1, 2, sp()),
        "wsum": lambda: _lib.wsum_ptrs(0, ptrs, w, p, out.data_ptr(), sp()),
    }
    for ch in (12, 16, 20, 116, 120):
        for grid in (0, 256 * 8):
            legs["bigtile_ch%d_grid%d" % (ch, grid)] = (
                lambda ch=ch, grid=grid: so.dlp_bigtile8(arr, wf, each, out.data_ptr(), ch, grid, sp()))
    res = {k: [] for k in legs}
    # the big-tile probe must produce the product's bits (same per-element fold order)
    _lib.wsum_ptrs(0, ptrs, w, p, out.data_ptr(), sp())
    ref = out.clone()
    so.dlp_bigtile8(arr, wf, each, out.data_ptr(), 16, 2048, sp())
    torch.cuda.synchronize()
    print(json.dumps({"bigtile_bit_exact": bool(torch.equal(ref.view(torch.int32), out.view(torch.int32)))}))
    for _ in range(5):
        for k, fn in legs.items():
            res[k].append(ev_time(fn))
    med = {k: statistics.median(v) for k, v in res.items()}
    gb = {"read8": 8 * each, "write_plain": each, "write_sc1": each}
    gb = {k: gb.get(k, 9 * each) for k in legs}
    for k in legs:
        print(json.dumps({"leg": k, "us": round(med[k], 2), "GB/s": round(gb[k] / med[k] / 1e3, 1)}))
    print(json.dumps({"read8 + write_sc1 (sequential sum)": round(med["read8"] + med["write_sc1"], 2),
                      "read8+w_sc1 (mixed)": round(med["read8+w_sc1"], 2), "wsum": round(med["wsum"], 2)}))


if __name__ == "__main__":
    main()
