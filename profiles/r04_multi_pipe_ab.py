"""r04: A/B legs of the many-tensor table kernel (dla_wsum_multi_table, device-resident module rounds;
VERDICT r03 next 3: 16 x ResNet-34 bf16 at 0.68 of peak), each leg one setting of a tuning-build
environment knob read per call:
  * DLA_MULTI_PIPE=0/2/4 (lib/ab/libdlagg_pipe.so): the one-block kernel against the software-
    pipelined variant (BLK blocks of 64 vectors per workgroup, block i+1's loads issued before block
    i's fold; one tensor lookup per BLK blocks);
  * DLA_MULTI_VW=2/4 (lib/ab/libdlagg_vw.so): 8-byte against 16-byte loads per lane (512 B against
    1 KiB of each peer per wave);
  * DLA_MULTI_WGS=W (lib/ab/libdlagg_wgs.so): an occupancy cap of W workgroups per CU (0 = none);
  * DLA_MULTI_G=8/16 (lib/ab/libdlagg_g.so): fold rounds of 8 peers for 9-32-peer passes, of 16 for
    larger passes, instead of 16 / 32 (0 = the product's).
Legs interleave in one process, HIP events on the launch stream, and every leg's output is compared
bit for bit with the first leg's.  Layouts: the reference models as
separate device tensors (tests/golden/layouts.json), at their BASELINE peer counts where a pass is
8 / 16 / 32 peers.
Usage on the GPU box: python profiles/r04_multi_pipe_ab.py [--lib PATH] [--knob DLA_MULTI_VW --values 2,4]
-> one JSON line per leg."""
import argparse
import ctypes
import json
import os
import statistics

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
vp, i64 = ctypes.c_void_p, ctypes.c_int64

SHAPES = {  # name: (layout, peers, dtype)
    "r34x16": ("google_speech_resnet34", 16, torch.bfloat16),
    "r34x32": ("google_speech_resnet34", 32, torch.bfloat16),
    "r8x16": ("cifar10_resnet8", 16, torch.float32),
    "r8x32": ("cifar10_resnet8", 32, torch.float32),
    "femx32": ("femnist_cnn", 32, torch.float32),
    "femx8": ("femnist_cnn", 8, torch.float32),
    "r34x128": ("google_speech_resnet34", 128, torch.bfloat16),
    "r8x64": ("cifar10_resnet8", 64, torch.float32),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "decentralized-learning_amd", "lib", "ab", "libdlagg_pipe.so"))
    ap.add_argument("--shapes", default="r34x16,r34x32,r8x16,r8x32,femx32,femx8")
    ap.add_argument("--knob", default="DLA_MULTI_PIPE")
    ap.add_argument("--values", default="0,2,4")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    so = ctypes.CDLL(os.path.abspath(args.lib))
    so.dla_wsum_multi_table.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                        ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double), ctypes.c_int, vp, vp, vp]
    so.dla_wsum_multi_table.restype = ctypes.c_int
    so.dla_wsum_multi_table_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    so.dla_wsum_multi_table_bytes.restype = i64
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    layouts = json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))
    for key in args.shapes.split(","):
        lay, n, dt = SHAPES[key]
        shapes = [s for _, s, _ in layouts[lay]["params"]]
        numels = [int(np.prod(s)) if s else 1 for s in shapes]
        base = torch.randn(sum(numels), device=dev) * 0.05
        peers = [[t.clone() for t in (base * (1.0 + 0.001 * k)).to(dt).split(numels)] for k in range(n)]
        t_n = len(numels)
        ptrs = (vp * (t_n * n))(*[peers[k][t].data_ptr() for t in range(t_n) for k in range(n)])
        nums = (i64 * t_n)(*numels)
        w = (ctypes.c_double * n)(*np.random.default_rng(n).dirichlet(np.ones(n)).tolist())
        nbytes = so.dla_wsum_multi_table_bytes(t_n, n)
        code = 0 if dt == torch.float32 else 1
        es = 4 if dt == torch.float32 else 2
        legs, outs = {}, {}
        values = args.values.split(",")
        for blk in values:
            o = [torch.empty(m, dtype=dt, device=dev) for m in numels]
            op = (vp * t_n)(*[x.data_ptr() for x in o])
            th = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            td = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            outs[blk] = o

            def fn(blk=blk, op=op, th=th, td=td):
                os.environ[args.knob] = blk
                rc = so.dla_wsum_multi_table(code, t_n, ptrs, op, nums, w, n, th.data_ptr(), td.data_ptr(), sp)
                if rc != 0:
                    raise RuntimeError("dla_wsum_multi_table rc=%d" % rc)
            legs[blk] = (fn, th, td)
        res = {b: [] for b in legs}
        for fn, _, _ in legs.values():
            for _ in range(5):
                fn()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for b, (fn, _, _) in legs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                fn()
                e0.record(stream)
                for _ in range(args.reps):
                    fn()
                e1.record(stream)
                e1.synchronize()
                res[b].append(e0.elapsed_time(e1) / args.reps * 1e3)
        byts = (n + 1) * sum(numels) * es
        for b in legs:
            same = all(torch.equal(x.view(torch.int16 if es == 2 else torch.int32),
                                   y.view(torch.int16 if es == 2 else torch.int32))
                       for x, y in zip(outs[b], outs[values[0]]))
            t = statistics.median(res[b])
            print(json.dumps({"shape": key, "peers": n, "tensors": t_n, args.knob: b,
                              "us": round(t, 2), "min_us": round(min(res[b]), 2), "GB/s": round(byts / t / 1e3, 1),
                              "frac_8TBs": round(byts / t / 1e3 / 8000, 4), "bit_exact_vs_first_leg": same}),
                  flush=True)
        del peers, outs, legs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
