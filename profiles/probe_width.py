"""r02 probes (csrc/probe.hip; diagnostics, not the product path), run on the GPU box:

  python profiles/probe_width.py              timing table: the many-peer access pattern of the
                                              word/vector-per-lane FedAvg kernels WITHOUT the
                                              arithmetic (128 rows x 5.32 MB = configs[4]'s
                                              per-GPU bf16 share), per load width and peers in
                                              flight, with and without the output write
  python profiles/probe_width.py --calib W    20 reads of a known 1 GiB buffer with W-byte loads
                                              (W = 4, 8, 16), for a rocprofv3 --pmc FETCH_SIZE
                                              pass: calibrates FETCH_SIZE for that load width
                                              (MI355X_MICROARCH.md: only 16-B reads are calibrated)
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
from accdfl_amd import _lib  # noqa: E402

so = ctypes.CDLL(_lib.build_probe())
vp = ctypes.c_void_p
so.dlp_read_width.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int, vp]
so.dlp_mread_width.argtypes = [vp, ctypes.c_int, ctypes.c_int64, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
so.dlp_mread_unrolled.argtypes = [vp, ctypes.c_int64, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64,
                                  vp]


def ev_time(fn, reps=30, warm=3):
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    sp = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    if len(sys.argv) > 2 and sys.argv[1] == "--calib":
        w = int(sys.argv[2])
        nbytes = 1 << 30
        buf = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).normal_()
        for _ in range(20):
            assert so.dlp_read_width(buf.data_ptr(), nbytes, sink.data_ptr(), w, sp()) == 0
        torch.cuda.synchronize()
        print(json.dumps({"calib_width": w, "bytes_per_dispatch": nbytes, "dispatches": 20}))
        return
    res = {}
    nbytes = 1 << 30
    buf = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).normal_()
    for w in (4, 8, 16):
        t = ev_time(lambda: so.dlp_read_width(buf.data_ptr(), nbytes, sink.data_ptr(), w, sp()))
        res["read_1GiB_w%d_GBps" % w] = round(nbytes / t / 1e9, 1)
    del buf
    n_src, each = 128, 2_662_045 * 2 // 16 * 16
    rows = torch.empty((n_src, each // 4), dtype=torch.float32, device=dev).normal_()
    dst = torch.empty(each // 4, dtype=torch.float32, device=dev)
    arr = (ctypes.c_void_p * n_src)(*[rows[k].data_ptr() for k in range(n_src)])
    for rnd in range(3):
        for w, g in ((4, 16), (4, 32), (4, 64), (8, 16), (8, 32), (16, 8), (16, 16)):
            for wr in (0, 1):
                t = ev_time(lambda: so.dlp_mread_width(arr, n_src, each, dst.data_ptr(), sink.data_ptr(), w, g, wr,
                                                       sp()))
                key = "mread128_w%d_g%d_write%d" % (w, g, wr)
                res.setdefault(key, []).append(round((n_src + wr) * each / t / 1e9, 1))
    # unrolled schedule (the FedAvg kernel's), row-major rows as above
    for rnd in range(3):
        for w, g in ((8, 16), (8, 32), (16, 16), (4, 64)):
            for wr in (0, 1):
                t = ev_time(lambda: so.dlp_mread_unrolled(arr, each, dst.data_ptr(), sink.data_ptr(), w, g, wr, 0,
                                                          sp()))
                res.setdefault("unrolled128_w%d_g%d_write%d" % (w, g, wr), []).append(
                    round((n_src + wr) * each / t / 1e9, 1))
    del rows
    # tile-interleaved layout: tile t of row k at base + (t * 128 + k) * tile_bytes
    for tile in (1024, 4096, 16384, 65536):
        n_t = -(-each // tile)
        slab = torch.empty(n_t * 128 * tile // 4, dtype=torch.float32, device=dev).normal_()
        tarr = (ctypes.c_void_p * n_src)(*[slab.data_ptr() + k * tile for k in range(n_src)])
        for rnd in range(3):
            for w, g in ((8, 16), (8, 32)):
                t = ev_time(lambda: so.dlp_mread_unrolled(tarr, each, dst.data_ptr(), sink.data_ptr(), w, g, 1,
                                                          tile, sp()))
                res.setdefault("interleaved%d_w%d_g%d_write1" % (tile, w, g), []).append(
                    round((n_src + 1) * each / t / 1e9, 1))
        del slab
    for k, v in res.items():
        print(json.dumps({k: v}))


if __name__ == "__main__":
    main()
