"""A short, fixed launch sequence for rocprofv3 counter passes (r03): `reps` launches of
dla_wsum_slab_tiled per shape from the library at --lib (default: the tree's), after a short
settle.  Shapes as profiles/ab_r03_kernels.py: ns (8 x 25 M f32, 16 KiB tiles), c4share
(128 x 2 662 045 bf16, 4 KiB tiles), c4whole (128 x 21 296 355 bf16, 4 KiB).
Device-module shapes (r04, VERDICT r03 next 3: wsum_multi_vec_kernel's counters): r34x16 / r34x128 —
16 / 128 google_speech ResNet-34 bf16 models as separate device tensors (the reference layout,
tests/golden/layouts.json) through wsum_multi_ptrs (dla_wsum_multi_table, one launch per pass).
Usage: rocprofv3 --pmc ... -- python3 profiles/pmc_driver.py [--lib PATH] ns,c4share"""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
sys.path.insert(0, os.path.join(ROOT, "profiles"))
from accdfl_amd import _lib  # noqa: E402
from ab_r03_kernels import bind_tiled  # noqa: E402

SHAPES = {"ns": (8, 25_000_000, torch.float32, 16384), "c4share": (128, 2_662_045, torch.bfloat16, 4096),
          "c4whole": (128, 21_296_355, torch.bfloat16, 4096),
          # round 5: the flat tile-interleaved slab of the same bytes as r34x16 (16 KiB tiles for 16 rows)
          "r34flat16": (16, 21_296_355, torch.bfloat16, 16384)}


MODULE_SHAPES = {"r34x16": ("google_speech_resnet34", 16), "r34x128": ("google_speech_resnet34", 128),
                 # round 6: the same models with each model's parameters as 256-byte
                 # aligned views of ONE allocation per model instead of one caching-allocator block each
                 "r34x16c": ("google_speech_resnet34", 16), "r34x128c": ("google_speech_resnet34", 128)}


def contiguous_model(numels, dtype, dev, shift_bytes=0):
    """One model's parameters as views of one allocation, each starting 256-byte aligned; with
    ``shift_bytes`` every view starts that many bytes (a multiple of 256) further into the allocation."""
    es = torch.tensor([], dtype=dtype).element_size()
    al = 256 // es
    offs, o = [], shift_bytes // es
    for m in numels:
        offs.append(o)
        o += -(-m // al) * al
    flat = torch.empty(max(o, 1), dtype=dtype, device=dev)
    return [flat[a:a + m] for a, m in zip(offs, numels)]


def module_round(key, reps, dev):
    import json

    import numpy as np

    from accdfl_amd.core import wsum

    lay, n = MODULE_SHAPES[key]
    shapes = [s for _, s, _ in json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))[lay]["params"]]
    numels = [int(np.prod(s)) if s else 1 for s in shapes]
    # separate allocations, uninitialised (no fill kernels: under --pmc every dispatch is serialised and
    # 14 080 fills would take minutes; the values do not change the reduce's timing or its traffic)
    if key.endswith("c"):
        peers = [contiguous_model(numels, torch.bfloat16, dev) for _ in range(n)]
    else:
        peers = [[torch.empty(m, dtype=torch.bfloat16, device=dev) for m in numels] for _ in range(n)]
    outs = [torch.empty(m, dtype=torch.bfloat16, device=dev) for m in numels]
    ptrs = (ctypes.c_void_p * (n * len(numels)))(*[peers[k][t].data_ptr() for t in range(len(numels))
                                                   for k in range(n)])
    out_p = (ctypes.c_void_p * len(numels))(*[o.data_ptr() for o in outs])
    nums = (ctypes.c_int64 * len(numels))(*numels)
    w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
    for _ in range(reps):
        wsum.wsum_multi_ptrs(torch.bfloat16, ptrs, out_p, nums, w, dev)
    torch.cuda.synchronize()
    print("%s: %d launches (%d tensors x %d peers)" % (key, reps, len(numels), n), flush=True)
    del peers, outs
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes")
    ap.add_argument("--lib", default="")
    ap.add_argument("--reps", type=int, default=40)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    so = bind_tiled(ctypes.CDLL(os.path.abspath(args.lib)) if args.lib else _lib.lib().so)
    sp = torch.cuda.current_stream(dev).cuda_stream
    for key in args.shapes.split(","):
        if key in MODULE_SHAPES:
            module_round(key, args.reps, dev)
            continue
        n, p, dt, tile_b = SHAPES[key]
        es = torch.tensor([], dtype=dt).element_size()
        te = tile_b // es
        slab = torch.empty(-(-p // te) * n * te, dtype=dt, device=dev).normal_(0, 0.05)
        out = torch.empty(p, dtype=dt, device=dev)
        wa = (ctypes.c_double * n)(*torch.distributions.Dirichlet(torch.ones(n)).sample().tolist())
        code = {torch.float32: 0, torch.bfloat16: 1}[dt]
        for _ in range(args.reps):
            rc = so.dla_wsum_slab_tiled(code, slab.data_ptr(), te, n, wa, n, p, out.data_ptr(), sp, None)
            if rc != 0:
                raise RuntimeError("dla_wsum_slab_tiled rc=%d" % rc)
        torch.cuda.synchronize()
        print("%s: %d launches" % (key, args.reps), flush=True)
        del slab, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
