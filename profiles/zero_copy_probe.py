"""Small-round host path, DMA vs zero-copy (diagnostic, GPU box).

The small-round path (fedavg._small_round: GNLeNet N=2 is the GL merge) packs the peers
into a pinned row, DMAs it H2D, launches the reduce, and DMAs the result back.  This probe
times that sequence against a "zero-copy" variant in which the reduce kernel reads the
pinned staging rows and writes the pinned result row directly over PCIe (device-mapped
host pointers from hipHostGetDevicePointer), and checks both bit-exact against each other.
Usage: python profiles/zero_copy_probe.py [N ...]"""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
import torch  # noqa: E402
from torch import nn  # noqa: E402

from accdfl_amd import _lib  # noqa: E402
from accdfl_amd.core.gradient_aggregation import fedavg as fa  # noqa: E402

SHAPES = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,), (64, 32, 5, 5), (64,), (64,),
          (64,), (10, 576), (10,)]
hip = ctypes.CDLL("libamdhip64.so")


def dev_ptr(host_ptr: int) -> int:
    out = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(out), ctypes.c_void_p(host_ptr), 0)
    if rc != 0:
        raise RuntimeError("hipHostGetDevicePointer failed: %d" % rc)
    return out.value


def t(fn, reps=400):
    for _ in range(30):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def run(n):
    torch.manual_seed(n)
    models = [nn.ParameterList([nn.Parameter(torch.randn(s) * 0.05) for s in SHAPES]) for _ in range(n)]
    w = [float(x) for x in torch.rand(n, dtype=torch.float64)]
    dev = torch.device("cuda", 0)
    numels = [torch.Size(s).numel() for s in SHAPES]
    total = sum(numels)
    pitch = (total + 63) // 64 * 64
    st = fa._HostStaging(dev, torch.float32)
    st.ensure(n, pitch)
    peers = [list(m.parameters()) for m in models]
    cur = torch.cuda.current_stream(dev)
    row_bytes = pitch * 4
    dsts, srcs, nb = [], [], []
    for k in range(n):
        off = st.h_in.data_ptr() + k * row_bytes
        for p in peers[k]:
            dsts.append(off)
            srcs.append(p.data_ptr())
            nb.append(p.numel() * 4)
            off += p.numel() * 4

    def pack():
        _lib.host_copy_batch(dsts, srcs, nb)

    def dma():
        st.d_in[:n].copy_(st.h_in[:n], non_blocking=True)
        st.plan_for(n, total, w).launch(int(cur.cuda_stream))
        st.h_out[:total].copy_(st.d_out[:total], non_blocking=True)
        cur.synchronize()

    h_zc = torch.empty(pitch, dtype=torch.float32, pin_memory=True)
    in_d = dev_ptr(st.h_in.data_ptr())
    out_d = dev_ptr(h_zc.data_ptr())
    zplan = _lib.Plan(0, [in_d + k * row_bytes for k in range(n)], w, total, out_d)

    def zc():
        zplan.launch(int(cur.cuda_stream))
        cur.synchronize()

    pack()
    dma()
    zc()
    exact = torch.equal(st.h_out[:total].view(torch.int32), h_zc[:total].view(torch.int32))
    res = {"n": n, "params": total, "bytes_in": n * total * 4, "bit_exact_zc_vs_dma": exact,
           "pack_us": t(pack), "dma_h2d_launch_d2h_sync_us": t(dma), "zero_copy_launch_sync_us": t(zc),
           "center_copy_us": t(lambda: fa._center_copy(models[0], pin=False)),
           "aggregate_us": t(lambda: fa.FedAvg.aggregate(models, w))}
    print(json.dumps(res), flush=True)
    if not exact:
        raise SystemExit("zero-copy result differs from the DMA path")


if __name__ == "__main__":
    for a in (sys.argv[1:] or ["2", "8"]):
        run(int(a))
