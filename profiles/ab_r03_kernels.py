"""r03 interleaved A/B on the tile-interleaved slab (dla_wsum_slab_tiled), one process:
  * the tree's libdlagg.so against a saved build (--base, default lib/ab/libdlagg_r03base.so), bit
    for bit on every shape;
  * the LDS-DMA probe of the north star (probe dlp_ldsdma_tiled8, S stages of 8 x 1 KiB
    global_load_lds_dwordx4 per wave, persistent one-wave workgroups) against the product kernel,
    bit for bit on the units it computes.
Shapes: the north star (8 x 25 M f32, 16 KiB tiles), configs[4]'s per-GPU share (128 x 2 662 045
bf16, 4 KiB), configs[4] whole (128 x 21 296 355 bf16, 4 KiB), 16 x 21.3 M bf16 (16 KiB).
Median over interleaved rounds of HIP-event time per launch (events on the launch stream)."""
import argparse
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

vp, i64 = ctypes.c_void_p, ctypes.c_int64


def bind_tiled(so):
    so.dla_wsum_slab_tiled.argtypes = [ctypes.c_int, vp, i64, i64, ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                                       i64, vp, vp, vp]
    so.dla_wsum_slab_tiled.restype = ctypes.c_int
    return so


def ev_time(fn, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us per launch


def settle(fn, seconds=0.2):
    t = time.time()
    while time.time() - t < seconds:
        for _ in range(20):
            fn()
        torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", default=os.path.join(ROOT, "decentralized-learning_amd", "lib", "ab", "libdlagg_r03base.so"))
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--shapes", default="ns,c4share,c4whole,b16")
    ap.add_argument("--stages", default="2,3,4,6")
    ap.add_argument("--grids", default="0")
    ap.add_argument("--ns-tiles", default="", help="extra tile sizes (bytes) for the north star, tree build")
    ap.add_argument("--variants", default="", help="extra tree legs with these launch variants (e.g. 8,12,28)")
    ap.add_argument("--auto-tile", action="store_true", help="tile every shape as PeerSlab does "
                                                                "(dla_slab_tile_elems) instead of its fixed tile")
    ap.add_argument("--no-ldsdma", action="store_true", help="skip the LDS-DMA probe legs of the north star")
    ap.add_argument("--rows", default="", help="also time the peers as separate row-major buffers: default + "
                                               "these dla_wsum_ex variants (e.g. 9,12)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    libs = {"tree": bind_tiled(_lib.lib().so)}
    if args.base and os.path.exists(args.base):
        libs["base"] = bind_tiled(ctypes.CDLL(os.path.abspath(args.base)))
    probe = None if args.no_ldsdma else ctypes.CDLL(_lib.build_probe())
    if probe is not None:
        probe.dlp_ldsdma_tiled8.argtypes = [vp, ctypes.POINTER(ctypes.c_float), i64, vp, ctypes.c_int, ctypes.c_int, vp]
        probe.dlp_ldsdma_tiled8.restype = ctypes.c_int
    shapes = {
        "ns": ("north star 8 x 25 M f32", 8, 25_000_000, torch.float32, 16384),
        "c4share": ("configs[4] share 128 x 2 662 045 bf16", 128, 2_662_045, torch.bfloat16, 4096),
        "c4whole": ("configs[4] whole 128 x 21 296 355 bf16", 128, 21_296_355, torch.bfloat16, 4096),
        "b16": ("16 x 21 296 355 bf16", 16, 21_296_355, torch.bfloat16, 16384),
        "c2": ("configs[2] 32 x 1 690 046 f32", 32, 1_690_046, torch.float32, 4096),
        "c3p": ("configs[3'] whole 64 x 4 932 344 f32", 64, 4_932_344, torch.float32, 4096),
        "ns4": ("4 x 25 M f32", 4, 25_000_000, torch.float32, 16384),
        "ns16": ("16 x 25 M f32", 16, 25_000_000, torch.float32, 16384),
        "b8": ("8 x 50 M bf16", 8, 50_000_000, torch.bfloat16, 16384),
        "ns2": ("2 x 25 M f32", 2, 25_000_000, torch.float32, 16384),
        "ns12": ("12 x 25 M f32", 12, 25_000_000, torch.float32, 16384),
        "ns6": ("6 x 25 M f32", 6, 25_000_000, torch.float32, 16384),
        "c3b": ("configs[3'] bucket 64 x 1 233 086 f32", 64, 1_233_086, torch.float32, 4096),
        "ns_2": ("north star share at N=2: 8 x 12.5 M f32", 8, 12_500_000, torch.float32, 16384),
        "ns_4": ("north star share at N=4: 8 x 6.25 M f32", 8, 6_250_000, torch.float32, 16384),
        "ns_8": ("north star share at N=8: 8 x 3.125 M f32", 8, 3_125_000, torch.float32, 16384),
    }
    g = torch.Generator(device="cpu").manual_seed(3)
    for key in args.shapes.split(","):
        if key.startswith("n") and key[1:].isdigit():  # nK: K peers x 25 M f32, 16 KiB tiles
            shapes[key] = ("%s x 25 M f32" % key[1:], int(key[1:]), 25_000_000, torch.float32, 16384)
        if key.startswith("p") and "x" in key:  # pKxM: K peers x M million f32, 4 KiB tiles
            k_, m_ = key[1:].split("x")
            shapes[key] = ("%s x %s M f32" % (k_, m_), int(k_), int(float(m_) * 1e6), torch.float32, 4096)
        name, n, p, dt, tile_b = shapes[key]
        es = torch.tensor([], dtype=dt).element_size()
        te = tile_b // es
        if args.auto_tile:
            te = _lib.slab_tile_elems({torch.float32: 0, torch.bfloat16: 1}[dt], n, p)
            name += " (%d KiB tiles)" % (te * es >> 10)
        n_t = -(-p // te)
        slab = torch.empty(n_t * n * te, dtype=dt, device=dev)
        slab.normal_(0, 0.05)
        w = torch.distributions.Dirichlet(torch.ones(n)).sample().tolist()
        wa = (ctypes.c_double * n)(*w)
        code = {torch.float32: 0, torch.bfloat16: 1}[dt]
        outs = {}
        legs = {}
        for lname, so in libs.items():
            o = torch.empty(p, dtype=dt, device=dev)
            outs[lname] = o

            def fn(so=so, o=o):
                rc = so.dla_wsum_slab_tiled(code, slab.data_ptr(), te, n, wa, n, p, o.data_ptr(), sp, None)
                if rc != 0:
                    raise RuntimeError("dla_wsum_slab_tiled rc=%d" % rc)
            legs[lname] = fn
        if args.rows:  # the same peers as separate row-major buffers (dla_wsum / dla_wsum_ex)
            pitch = -(-p // 64) * 64
            rows = torch.empty(n, pitch, dtype=dt, device=dev)
            rows[:, :p].copy_(slab[: n_t * n * te].view(n_t, n, te).permute(1, 0, 2).reshape(n, -1)[:, :p])
            rptrs = [rows[k].data_ptr() for k in range(n)]
            for v in [0] + [int(x) for x in args.rows.split(",") if x]:
                o = torch.empty(p, dtype=dt, device=dev)
                lname = "rows v%d" % v if v else "rows default"
                outs[lname] = o

                def fn(v=v, o=o, rows=rows, rptrs=rptrs):
                    _lib.wsum_ptrs(code, rptrs, w, p, o.data_ptr(), sp, _lib.LaunchCfg(v, 0, 0, 0) if v else None)
                legs[lname] = fn
        for v in [int(x) for x in args.variants.split(",") if x]:
            cfg = _lib.LaunchCfg(v, 0, 0, 0)
            o = torch.empty(p, dtype=dt, device=dev)
            lname = "tree v%d" % v
            outs[lname] = o

            def fn(cfg=cfg, o=o):
                rc = libs["tree"].dla_wsum_slab_tiled(code, slab.data_ptr(), te, n, wa, n, p, o.data_ptr(), sp,
                                                      ctypes.byref(cfg))
                if rc != 0:
                    raise RuntimeError("dla_wsum_slab_tiled rc=%d" % rc)
            legs[lname] = fn
        if args.ns_tiles:  # re-tiled copies of the same peers (any shape)
            for tb in [int(x) for x in args.ns_tiles.split(",")]:
                t2 = tb // es
                sl2 = torch.empty(-(-p // t2) * n * t2, dtype=dt, device=dev)
                # the same peers, re-tiled: peer k's element i at ((i // t2) * n + k) * t2 + i % t2
                src = slab[: n_t * n * te].view(n_t, n, te).permute(1, 0, 2).reshape(n, -1)[:, :p]
                full = -(-p // t2) * t2
                pad = torch.zeros(n, full, dtype=dt, device=dev)
                pad[:, :p] = src
                sl2.copy_(pad.view(n, -1, t2).permute(1, 0, 2).reshape(-1))
                del pad, src
                o = torch.empty(p, dtype=dt, device=dev)
                lname = "tree tile %d B" % tb
                outs[lname] = o

                def fn(sl2=sl2, t2=t2, o=o):
                    rc = libs["tree"].dla_wsum_slab_tiled(code, sl2.data_ptr(), t2, n, wa, n, p, o.data_ptr(), sp,
                                                          None)
                    if rc != 0:
                        raise RuntimeError("dla_wsum_slab_tiled rc=%d" % rc)
                legs[lname] = fn
        if key == "ns" and not args.no_ldsdma:
            w8 = (ctypes.c_float * 8)(*[float(torch.tensor(x, dtype=torch.float32)) for x in w])
            for s in [int(x) for x in args.stages.split(",") if x]:
                for gr in [int(x) for x in args.grids.split(",")]:
                    o = torch.zeros(p, dtype=dt, device=dev)
                    lname = "ldsdma S=%d grid=%s" % (s, gr or "auto")
                    outs[lname] = o

                    def fn(s=s, gr=gr, o=o):
                        rc = probe.dlp_ldsdma_tiled8(slab.data_ptr(), w8, p, o.data_ptr(), s, gr, sp)
                        if rc != 0:
                            raise RuntimeError("dlp_ldsdma_tiled8 rc=%d" % rc)
                    legs[lname] = fn
        for fn in legs.values():
            settle(fn)
        res = {k: [] for k in legs}
        for _ in range(args.rounds):
            for k, fn in legs.items():
                res[k].append(ev_time(fn, args.reps, stream))
        torch.cuda.synchronize()
        ref = outs["tree"]
        byts = (n + 1) * p * es
        for k in legs:
            o = outs[k]
            cover = p if not k.startswith("ldsdma") else p // 256 * 256
            same = bool(torch.equal(o[:cover].view(torch.int16 if es == 2 else torch.int32),
                                    ref[:cover].view(torch.int16 if es == 2 else torch.int32)))
            t = statistics.median(res[k])
            print(json.dumps({"shape": name, "leg": k, "us": round(t, 2), "min_us": round(min(res[k]), 2),
                              "GB/s": round(byts / t / 1e3, 1), "frac_8TBs": round(byts / t / 1e3 / 8000, 4),
                              "bit_exact_vs_tree": same}), flush=True)
        del slab, outs, legs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
