"""r02: where a small round of CPU-resident models (the GL merge of N=2 GNLeNet models,
accdfl/gl/community.py:117; DFL N=8) spends its time on the GPU box, and the two ways of
moving it: the DMA round trip (pack into page-locked rows -> one H2D -> prepared launch -> one
D2H -> unpack; the r02 small path before dla_host_round_*, restated below) against the kernel reading the page-locked rows and writing
the page-locked result across PCIe (dla_host_round_start / dla_host_round_finish)."""
import json
import os
import statistics
import sys
import time

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
import bench  # noqa: E402
from accdfl_amd import _lib  # noqa: E402
from accdfl_amd.core.gradient_aggregation import fedavg as F  # noqa: E402


def med(fn, reps=300):
    for _ in range(10):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


def dma_round_trip(dev, n, peers, w, numels, total, pitch, rows, result, d_in, d_out, plan, center):
    """pack (dla_host_copy_batch) -> one H2D -> prepared launch -> one D2H -> unpack."""
    esize = 4
    dsts, srcs, nbytes = [], [], []
    for k in range(n):
        off = rows.data_ptr() + k * pitch * esize
        for p in peers[k]:
            dsts.append(off)
            srcs.append(p.data_ptr())
            nbytes.append(p.numel() * esize)
            off += p.numel() * esize
    _lib.host_copy_batch(dsts, srcs, nbytes)
    cs = torch.cuda.current_stream(dev)
    d_in[:n].copy_(rows[:n], non_blocking=True)
    plan.launch(int(cs.cuda_stream))
    result[:total].copy_(d_out[:total], non_blocking=True)
    cs.synchronize()
    src = result.data_ptr()
    dsts, srcs, nbytes = [], [], []
    for c, m in zip(center, numels):
        dsts.append(c.data_ptr())
        srcs.append(src)
        nbytes.append(m * esize)
        src += m * esize
    _lib.host_copy_batch(dsts, srcs, nbytes)


def models_of(n, numel):
    if numel is None:
        return bench._gnlenet_models(n)
    g = torch.Generator().manual_seed(n)
    return [nn.ParameterList([nn.Parameter(torch.randn(numel, generator=g))]) for _ in range(n)]


def main():
    res = {}
    dev = torch.device("cuda", 0)
    for name, n, numel in (("gnlenet_n2", 2, None), ("gnlenet_n8", 8, None), ("n8_1M", 8, 1 << 20),
                           ("n8_2M", 8, 2 << 20), ("n4_3.9M", 4, 3_900_000)):
        ms = models_of(n, numel)
        w = [1.0 / n] * n
        peers = [list(m.parameters()) for m in ms]
        numels = [p.numel() for p in peers[0]]
        total = sum(numels)
        pitch = F._round_up(total, 64)
        center = [torch.empty_like(p) for p in peers[0]]
        rows = torch.empty((n, pitch), pin_memory=True)
        result = torch.empty(pitch, pin_memory=True)
        ptrs = [p.data_ptr() for pl in peers for p in pl]
        outs = [c.data_ptr() for c in center]
        cs = torch.cuda.current_stream(dev).cuda_stream
        d_in = torch.empty((n, pitch), device=dev)
        d_out = torch.empty(pitch, device=dev)
        plan = _lib.Plan(0, [d_in[k].data_ptr() for k in range(n)], w, total, d_out.data_ptr())
        dma = lambda: dma_round_trip(dev, n, peers, w, numels, total, pitch, rows, result, d_in, d_out,  # noqa
                                     plan, center)

        def zero_copy():
            _lib.host_round_start(0, n, ptrs, numels, w, rows.data_ptr(), pitch, result.data_ptr(), cs)
            _lib.host_round_finish(0, numels, result.data_ptr(), outs, cs)

        r = {
            "aggregate_us": med(lambda: F.FedAvg.aggregate(ms, w)),
            "center_copy_us": med(lambda: F._center_copy(ms[0], large=False)),
            "parameters_lists_us": med(lambda: [list(m.parameters()) for m in ms]),
            "dma_round_trip_us": med(dma),
            "zero_copy_round_trip_us": med(zero_copy),
        }
        zero_copy()
        got = torch.cat([c.reshape(-1) for c in center]).clone()
        dma()
        want = torch.cat([c.reshape(-1) for c in center])
        r["same_bits"] = bool(torch.equal(got.view(torch.int32), want.view(torch.int32)))
        r["input_MB"] = round(n * total * 4 / 1e6, 2)
        res[name] = r
        print(json.dumps({name: r}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
