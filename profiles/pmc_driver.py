"""A short, fixed launch sequence for rocprofv3 counter passes (r03): `reps` launches of
dla_wsum_slab_tiled per shape from the library at --lib (default: the tree's), after a short
settle.  Shapes as profiles/ab_r03_kernels.py: ns (8 x 25 M f32, 16 KiB tiles), c4share
(128 x 2 662 045 bf16, 4 KiB tiles), c4whole (128 x 21 296 355 bf16, 4 KiB).
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
          "c4whole": (128, 21_296_355, torch.bfloat16, 4096)}


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
