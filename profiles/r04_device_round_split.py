"""r04: the host work of one device-resident module round, step by step (end to end
<= the reduce + 0.15 ms).  For 16 and 128 google_speech ResNet-34 bf16 models (bench.py's
device_module_configs layout): the median host time of every step fedavg._device_round takes, each
timed alone (the stream synchronised outside the timed region), then the end-to-end median of
FedAvg.aggregate under each group schedule in SCHEDULES (interleaved, the result checked bit-exact
against the first schedule's).
Usage on the GPU box: python profiles/r04_device_round_split.py -> JSON lines."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from accdfl_amd import _lib  # noqa: E402
from accdfl_amd.core import wsum as _wsum  # noqa: E402
from accdfl_amd.core.gradient_aggregation import fedavg as fa  # noqa: E402


def host_us(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    return round(statistics.median(ts) * 1e6, 1)


def e2e_ms(fn, reps=60):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3


def fixed32(n):
    return [(a, min(a + 32, n)) for a in range(0, n, 32)]


def first16(n):
    """16 models, then groups of 32, a tail under 32 joining the last."""
    out, a = [(0, min(16, n))], min(16, n)
    while a < n:
        b = n if n - a < 64 else a + 32
        out.append((a, b))
        a = b
    return out


def geometric(first, growth):
    def bounds(n):
        out, a, g = [], 0, first
        while a < n:
            b = n if n - a - g < g else a + g
            out.append((a, b))
            a, g = b, g * growth
        return out
    return bounds


# name -> (group bounds, smallest grouped round); "default" is fedavg's own _group_bounds
SCHEDULES = {"default": (None, 64), "single_launch": (fixed32, 1 << 30), "fixed32": (fixed32, 64),
             "first16_then32": (first16, 64), "first8_x2": (geometric(8, 2), 64), "first16_x2": (geometric(16, 2), 64),
             "first32_x3": (geometric(32, 3), 64)}


def split(models, w):
    mod = _lib.walk_module()
    row = {"peers": len(models)}
    row["layout"] = host_us(lambda: fa._device_layout(models))
    row["tensors_m0"] = host_us(lambda: mod.tensors(models[0], fa._PLAIN_SET))
    dtype, device, numels, table = fa._device_layout(models)
    p0, b0 = mod.tensors(models[0], fa._PLAIN_SET)
    row["param_type_check"] = host_us(lambda: any(type(p) is not torch.nn.Parameter for p in p0))
    offs, total, byte_offs, nums = fa._flat_plan(dtype, numels)
    row["flat_plan"] = host_us(lambda: fa._flat_plan(dtype, numels))
    row["empty"] = host_us(lambda: torch.empty(total, dtype=dtype, device=device))
    flat = torch.empty(total, dtype=dtype, device=device)
    ptrs = (ctypes.c_void_p * table.size).from_buffer(table)
    outs = (ctypes.c_void_p * len(numels)).from_buffer(byte_offs + flat.data_ptr())
    row["ctypes_tables"] = host_us(lambda: ((ctypes.c_void_p * table.size).from_buffer(table),
                                           (ctypes.c_void_p * len(numels)).from_buffer(byte_offs + flat.data_ptr())))
    row["launch"] = host_us(lambda: _wsum.wsum_multi_ptrs(dtype, ptrs, outs, nums, w, device))
    row["param_views"] = host_us(lambda: mod.param_views(flat, p0, offs, {}))
    row["buffer_copies"] = host_us(lambda: mod.buffer_copies(b0, {}))
    pm = {}
    mod.param_views(flat, p0, offs, pm)
    row["seed_buffers"] = host_us(lambda: fa._seed_buffers(b0, dict(pm)))
    bdt = max({b.dtype for b in b0}, key=lambda d: sum(b.dtype == d for b in b0))
    bfl = [b for b in b0 if b.dtype == bdt]
    cfl = [torch.empty_like(b) for b in bfl]
    row["foreach_copy_%s" % str(bdt).replace("torch.", "")] = host_us(lambda: torch._foreach_copy_(cfl, bfl))
    memo = dict(pm)
    fa._seed_buffers(b0, memo)
    for native in (False, True):
        fa._NATIVE_CLONE = native
        row["clone_tree_" + ("native" if native else "python")] = host_us(lambda: fa._clone_value(models[0], dict(memo)))
    row["memo_copy"] = host_us(lambda: dict(memo))
    row["device_round"] = host_us(lambda: fa._device_round(models, w, (dtype, device, numels, table)))
    row["aggregate_no_sync"] = host_us(lambda: fa.FedAvg.aggregate(models, w))
    return row


def timeline(models, w, reps=20):
    """Host time of each launch of a grouped round and the GPU time between them (events recorded on the
    launch stream after each wsum_multi_ptrs call), medians over reps: where the GPU waits on the walk."""
    real = _wsum.wsum_multi_ptrs
    marks = []

    def traced(*a, **k):
        r = real(*a, **k)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks.append((time.perf_counter(), ev, sum(1 for _ in a[4])))
        return r

    rows = []
    _wsum.wsum_multi_ptrs = traced
    try:
        for _ in range(reps):
            marks.clear()
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            t0 = time.perf_counter()
            fa.FedAvg.aggregate(models, w)
            t_ret = time.perf_counter()
            torch.cuda.synchronize()
            t_end = time.perf_counter()
            rows.append([(round((t - t0) * 1e3, 4), round(e0.elapsed_time(ev), 4), n) for t, ev, n in marks]
                        + [("return", round((t_ret - t0) * 1e3, 4), "sync", round((t_end - t0) * 1e3, 4))])
    finally:
        _wsum.wsum_multi_ptrs = real
    mid = sorted(rows, key=lambda r: r[-1][-1])[len(rows) // 2]
    return {"peers": len(models), "schedule": [list(x) for x in mid],
            "legend": "per launch: [host ms after the call, GPU ms at the event after it, models]; then the return and sync times"}


def main():
    dev = torch.device("cuda", 0)
    default_bounds = fa._group_bounds
    for k, (fn, gmin) in list(SCHEDULES.items()):
        SCHEDULES[k] = (fn or default_bounds, gmin)
    for n in (16, 64, 128):
        models, _ = bench._device_layout_models("google_speech_resnet34", n, torch.bfloat16, dev)
        w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
        if n in (16, 128):
            print(json.dumps(split(models, w)), flush=True)
        for name, (fn, gmin) in SCHEDULES.items():
            fa._group_bounds, fa._GROUP_MIN = fn, gmin
            print(json.dumps(dict(timeline(models, w), name=name)), flush=True)
        fa._group_bounds, fa._GROUP_MIN = default_bounds, fa._GROUP_MIN_DEFAULT
        ref = None
        times = {k: [] for k in SCHEDULES}
        for it in range(6):
            for name, (fn, gmin) in SCHEDULES.items():
                fa._group_bounds = fn
                fa._GROUP_MIN = gmin
                out = fa.FedAvg.aggregate(models, w)
                flat = torch.cat([p.detach().reshape(-1) for p in out.parameters()]).view(torch.int16)
                if ref is None:
                    ref = flat
                elif not torch.equal(ref, flat):
                    raise SystemExit("schedule %s: result bits differ" % name)
                times[name].append(e2e_ms(lambda: fa.FedAvg.aggregate(models, w), reps=20))
        fa._group_bounds = default_bounds
        fa._GROUP_MIN = fa._GROUP_MIN_DEFAULT
        print(json.dumps({"peers": n, "e2e_ms": {k: [round(min(v), 4), round(statistics.median(v), 4)]
                                                  for k, v in times.items()}, "bit_exact": True}), flush=True)
        del models
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
