"""Round 6: where a device-resident FedAvg.aggregate round spends its time — 16 google_speech ResNet-34 bf16
device models (110 parameters, 108 BN buffers each), the steps of fedavg._device_round timed one by one on
the host (no synchronisation between them, as the product runs them), medians of 100 rounds:
  layout       — fedavg._device_layout (the native walk over every model: shapes, dtype, pointers);
  tensors      — walk.cpp tensors (models[0]'s parameter and buffer lists);
  blocks       — the result's parameters' caching-allocator blocks (walk.cpp param_blocks);
  launch       — dla_wsum_multi_table's host call (table upload + kernel launch);
  wrap         — their nn.Parameter objects in the deepcopy memo (walk.cpp param_wrap), while the reduce runs;
  buffers      — walk.cpp buffer_copies (models[0]'s buffers, one block each + one fused copy);
  clone        — the module tree's containers (_clone_value);
  wait         — torch.cuda.synchronize() after the clone: the GPU time not hidden behind the host steps;
plus the reduce alone (HIP events, back to back) and the whole FedAvg.aggregate call + synchronize; and, interleaved
round by round, the whole sequence with the parameters made in one step before the launch (param_fresh, the
round-6 form before param_blocks / param_wrap) against the two-step form."""
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "decentralized-learning_amd")]
import bench  # noqa: E402


def main():
    from accdfl_amd import _lib
    from accdfl_amd.core import wsum as _wsum
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    dev = torch.device("cuda", 0)
    mod = _lib.walk_module()
    n = 16
    if "--tree" in sys.argv:  # the reference's module tree (97 modules) instead of one ParameterList
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from test_center_copy_layouts import tree_from_layout

        models = []
        for k in range(n):
            t = tree_from_layout("google_speech_resnet34").to(torch.bfloat16)
            with torch.no_grad():
                for q in t.parameters():
                    q.copy_(torch.randn(q.shape, generator=torch.Generator().manual_seed(k)) * 0.05)
            models.append(t.to(dev))
    else:
        models, p = bench._device_layout_models("google_speech_resnet34", n, torch.bfloat16, dev)
    w = [float(x) for x in np.random.default_rng(1).dirichlet(np.ones(n))]
    for _ in range(5):
        fa.FedAvg.aggregate(models, w)
    torch.cuda.synchronize()
    keys = ("layout", "tensors", "blocks", "launch", "wrap", "buffers", "clone", "wait")
    split = {k: [] for k in keys}
    split["host"] = []
    results = []
    for _ in range(100):
        t = [time.perf_counter()]
        lay = fa._device_layout(models)
        t.append(time.perf_counter())
        dtype, device, numels, table = lay
        p0, b0 = mod.tensors(models[0], fa._PLAIN_SET)
        t.append(time.perf_counter())
        memo = {}
        blocks, out_ptrs = mod.param_blocks(p0)
        outs = (ctypes.c_void_p * len(numels)).from_buffer(out_ptrs)
        t.append(time.perf_counter())
        nums = fa._flat_plan(dtype, numels)[3]
        _wsum.wsum_multi_ptrs(dtype, (ctypes.c_void_p * table.size).from_buffer(table), outs, nums, w, device,
                              total_elems=sum(numels))
        t.append(time.perf_counter())
        mod.param_wrap(blocks, p0, memo)
        t.append(time.perf_counter())
        fa._seed_buffers(b0, memo)
        t.append(time.perf_counter())
        res = fa._clone_value(models[0], memo)
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        for k, a, b in zip(keys, t, t[1:]):
            split[k].append(b - a)
        split["host"].append(t[-2] - t[0])
        results.append(res)
        if len(results) > 4:
            results.pop(0)
    out = {k: round(statistics.median(v) * 1e6, 1) for k, v in split.items()}
    want = fa.FedAvg.aggregate(models, w)
    out["same_bits_as_aggregate"] = all(torch.equal(a.view(torch.int16), b.view(torch.int16))
                                        for a, b in zip(results[-1].parameters(), want.parameters()))
    # the reduce alone, back to back on the walked layout
    dtype, device, numels, table = fa._device_layout(models)
    outs_t = [torch.empty(k, dtype=dtype, device=dev) for k in numels]
    outs = (ctypes.c_void_p * len(numels))(*[o.data_ptr() for o in outs_t])
    nums = fa._flat_plan(dtype, numels)[3]
    ptrs = (ctypes.c_void_p * table.size).from_buffer(table)
    for _ in range(5):
        _wsum.wsum_multi_ptrs(dtype, ptrs, outs, nums, w, device, total_elems=sum(numels))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        _wsum.wsum_multi_ptrs(dtype, ptrs, outs, nums, w, device, total_elems=sum(numels))
    e1.record()
    torch.cuda.synchronize()
    out["reduce_us"] = round(e0.elapsed_time(e1) * 1e3 / 50, 1)
    ts = []
    for _ in range(100):
        t0 = time.perf_counter()
        fa.FedAvg.aggregate(models, w)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    out["aggregate_us"] = round(statistics.median(ts) * 1e6, 1)

    def seq(two_step):
        t0 = time.perf_counter()
        dtype, device, numels, table = fa._device_layout(models)
        p0, b0 = mod.tensors(models[0], fa._PLAIN_SET)
        memo = {}
        if two_step:
            blocks, out_ptrs = mod.param_blocks(p0)
        else:
            out_ptrs = mod.param_fresh(p0, memo)
        outs = (ctypes.c_void_p * len(numels)).from_buffer(out_ptrs)
        _wsum.wsum_multi_ptrs(dtype, (ctypes.c_void_p * table.size).from_buffer(table), outs,
                              fa._flat_plan(dtype, numels)[3], w, device, total_elems=sum(numels))
        if two_step:
            mod.param_wrap(blocks, p0, memo)
        fa._seed_buffers(b0, memo)
        res = fa._clone_value(models[0], memo)
        torch.cuda.synchronize()
        return time.perf_counter() - t0, res
    ab = {False: [], True: []}
    for _ in range(100):
        for two in (False, True):
            ab[two].append(seq(two)[0])
    out["one_step_us"] = round(statistics.median(ab[False]) * 1e6, 1)
    out["two_step_us"] = round(statistics.median(ab[True]) * 1e6, 1)
    out["n_models"], out["n_parameters"] = n, len(numels)
    out["n_buffers"] = len(mod.tensors(models[0], fa._PLAIN_SET)[1])
    out["n_modules"] = len(list(models[0].modules()))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
