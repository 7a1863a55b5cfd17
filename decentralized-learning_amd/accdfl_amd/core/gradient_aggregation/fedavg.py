"""FedAvg on MI355X — drop-in for accdfl/core/gradient_aggregation/fedavg.py:10-26.

``FedAvg.aggregate(models, weights)`` keeps the reference contract exactly:

* falsy ``weights`` -> uniform ``float(1. / N)`` (fedavg.py:14-15); otherwise
  ``assert len(weights) == len(models)`` (:16-17); empty ``models`` -> IndexError
  from ``models[0]`` (:20);
* the result is ``copy.deepcopy(models[0])`` (:20), so it lives where models[0]
  lives, keeps ``requires_grad`` and every non-parameter attribute, and carries
  models[0]'s buffers unaveraged;
* parameter i is ``R(...R(R(p0*0) + R(w0*p0)) + ... + R(w_{N-1}*p_{N-1}))`` in list
  order, bit-identical to the reference (fedavg.py:21-25; include/dlagg.h);
* zip truncation (:24): parameter i only takes terms from models that have an i-th
  parameter;
* models whose parameters have other dtypes than models[0]'s follow the reference's
  promotion (:25: the product rounded in the peer's dtype, the sum in models[0]'s);
* inputs are never mutated.

Deliberate difference (documented in DESIGN.md): parameters whose shapes differ between
models raise RuntimeError instead of broadcasting.

The result's CPU parameters are ordinary pageable tensors as in the reference; those of a
large round come from a pool of already-faulted pageable blocks (``core/host_memory.py``:
ACCDFL_AMD_RESULT_MEMORY=pooled, the default; "pinned" allocates them page-locked, which
keeps them page-locked for good; "pageable" allocates them fresh).

Where the arithmetic runs: always on the HIP device (libdlagg.so).  Models already
on the device are reduced in place of their parameters with no copies; models on several
GPUs are bucket-sharded over those GPUs (dla_wsum_sharded).  CPU models (every reference
call site): small rounds (_is_small: rows of at most _SMALL_ROW_BYTES = 64 MiB and under
_SMALL_ROUND_BYTES = 48 MiB of input in all, e.g. the GL merge of two models of any BASELINE
layout) are packed into page-locked rows that the kernel reads across PCIe
(dla_host_round_start / _finish) while the result module is built; larger rounds stream element
chunks through the GPU in one
native call (dla_host_reduce: a threaded pack of every peer's chunk into page-locked rows, one
DMA per chunk, the reduce, the D2H and the unpack into the result, two chunks in flight),
optionally bucket-sharded over several GPUs.  The host-staged paths are synchronous like the reference;
the device-resident path is stream-ordered like any torch op.
"""
from __future__ import annotations

import copy
import copyreg
import ctypes
import os
import threading
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch
from torch import nn

from accdfl_amd import _lib
from accdfl_amd.core import host_memory as _host_memory
from accdfl_amd.core import wsum as _wsum
from accdfl_amd.core.gradient_aggregation import GradientAggregation

_ALIGN_BYTES = 256


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class _HostStaging:
    """Pinned host slab + device slab for CPU-resident models, grown on demand and
    reused across calls (one per (device, dtype))."""

    def __init__(self, device: torch.device, dtype: torch.dtype):
        self.device = device
        self.dtype = dtype
        self.rows = 0
        self.pitch = 0
        self.h_in = self.d_in = self.d_out = self.h_out = None
        self.copy_stream = torch.cuda.Stream(device)
        self.plan = None       # prepared launch over (d_in rows, d_out), see _plan_for
        self.plan_key = None

    def ensure(self, rows: int, pitch: int):
        if rows <= self.rows and pitch <= self.pitch:
            return
        rows = max(rows, self.rows)
        pitch = max(pitch, self.pitch)
        self.h_in = torch.empty((rows, pitch), dtype=self.dtype, pin_memory=True)
        self.d_in = torch.empty((rows, pitch), dtype=self.dtype, device=self.device)
        self.d_out = torch.empty(pitch, dtype=self.dtype, device=self.device)
        self.h_out = torch.empty(pitch, dtype=self.dtype, pin_memory=True)
        self.rows, self.pitch = rows, pitch
        self.plan = self.plan_key = None

    def plan_for(self, n: int, total: int, weights) -> "_lib.Plan":
        """The prepared dla_plan for rows 0..n-1 of d_in -> d_out (cached across calls)."""
        key = (n, total, self.d_in.data_ptr(), self.d_out.data_ptr())
        if self.plan_key != key:
            ptrs = [self.d_in.data_ptr() + k * self.pitch * self.d_in.element_size() for k in range(n)]
            self.plan = _lib.Plan(_wsum.dtype_code(self.dtype), ptrs, weights, total, self.d_out.data_ptr())
            self.plan_key = key
        else:
            self.plan.set_weights(weights)
        return self.plan


_staging: Dict[Tuple[torch.device, torch.dtype], _HostStaging] = {}
_staging_lock = threading.Lock()


def _get_staging(device: torch.device, dtype: torch.dtype) -> _HostStaging:
    key = (device, dtype)
    st = _staging.get(key)
    if st is None:
        st = _staging[key] = _HostStaging(device, dtype)
    return st


_staging_sharded: Dict[Tuple[torch.device, torch.dtype, int], _HostStaging] = {}


def _get_staging_sharded(device: torch.device, dtype: torch.dtype, slot: int) -> _HostStaging:
    """Staging for bucket ``slot`` of a sharded reduce (distinct even when two buckets share a
    device, which the single-GPU tests use to exercise the sharded path)."""
    key = (device, dtype, slot)
    st = _staging_sharded.get(key)
    if st is None:
        st = _staging_sharded[key] = _HostStaging(device, dtype)
    return st


def release_staging() -> None:
    """Free the cached host/device staging slabs."""
    with _staging_lock:
        _staging.clear()
        _staging_sharded.clear()
        _native_staging.clear()
        _host_rounds.clear()


# Devices the host-staged path may shard over (one process, several GPUs): the reference
# hands CPU modules to the aggregator, so the path is PCIe-bound, and splitting the flat
# parameter vector into buckets sends each GPU's share over its own PCIe link.  Buckets keep
# every element's summation order: the result is bit-identical for any device count.
_host_devices: List[torch.device] = []
_MIN_SHARD_BYTES = 8 << 20  # per device; smaller models stay on one GPU


def set_host_devices(devices) -> None:
    """Use these HIP devices for CPU-resident models (an empty list restores the default: see
    _devices_for)."""
    global _host_devices
    _host_devices = [torch.device("cuda", d) if isinstance(d, int) else torch.device(d) for d in devices]


def _devices_for(device: torch.device, round_bytes: int = 0) -> List[torch.device]:
    """The GPUs a host-staged round of CPU models streams through, in bucket order:
    * set_host_devices([...]), else ACCDFL_AMD_DEVICES: a comma list of device ids, "all" (every
      visible GPU, the current one first: each bucket crosses its own GPU's PCIe link,
      bit-identically) or "current";
    * by default only the current device.  The reference runs every DFL / GL peer as its own ipv8
      process, so an aggregator that spread its rounds over every visible GPU would open a context,
      page-locked staging and HBM staging on GPUs other processes own and compete for their PCIe
      links: the several-GPU host path is opt-in.  The caller trims the list to the
      round's size (_MIN_SHARD_BYTES per device)."""
    if _host_devices:
        return list(_host_devices)
    env = os.environ.get("ACCDFL_AMD_DEVICES", "").strip().lower()
    if env and env not in ("all", "current"):
        return [torch.device("cuda", int(x)) for x in env.split(",") if x.strip()]
    if env != "all" or round_bytes < 2 * _MIN_SHARD_BYTES:
        return [device]
    count = torch.cuda.device_count()
    if count < 2:
        return [device]
    return [device] + [torch.device("cuda", d) for d in range(count) if d != device.index]


def _flat_slices(tensors: List[torch.Tensor], numels: List[int], start: int, end: int) -> List[torch.Tensor]:
    """1-D views covering [start, end) of the virtual concatenation of ``tensors``."""
    out, off = [], 0
    for t, n in zip(tensors, numels):
        s, e = max(start, off), min(end, off + n)
        if s < e:
            out.append(t.reshape(-1)[s - off:e - off])
        off += n
        if off >= end:
            break
    return out


# Small rounds go through dla_host_round_* (one native call packs every peer into page-locked rows
# and enqueues the reduce, which reads them across PCIe; one call waits and unpacks) instead of the
# chunked dla_host_reduce: below ~40 MB of input the one-shot round is faster (no per-chunk round
# trips); from ~50 to ~80 MB the two TIE within run-to-run noise, and the 48 MiB bound sits in that
# tie.  Round 4, both paths reading page-locked rows with the kernel, ms small / chunked, pageable
# peers — the re-run (profiles/r04s3/small_large_ab.jsonl): GNLeNet 8 peers 0.158 / 0.165, 64 peers
# (21.9 MB) 0.580 / 0.680; FEMNIST 2 peers 0.506 / 0.582, 4 peers (27 MB) 0.874 / 1.001, 8 peers
# (54 MB) 1.504 / 1.492 (tie); ResNet-8 2 peers (39.5 MB) 1.341 / 1.644, 4 peers (79 MB) 2.324 / 2.298
# (tie).  The first run (profiles/r04s2) read FEMNIST 8 peers 1.884 / 1.493 and GNLeNet 8 peers
# 0.160 / 0.154: single samples, not reproduced.  Round 2 (staging DMAs then), us
# small / dla_host_reduce (profiles/r02zo_layout_paths.log): FEMNIST 2 peers 619 / 828, 4 peers
# 943 / 1343, 8 peers (54 MB) 1644-1882 / 1759-1979, 32 peers (216 MB) 6152 / 4704; ResNet-8 2 peers
# 1393-2496 / 2290-2780, 3 peers 1895 / 2587, 4 peers (79 MB) 2497 / 2966, 8 peers (158 MB)
# 4951 / 4213; GNLeNet 8 peers 257 / 367, 64 peers 1084 / 1528.  (Round 2 first bounded it at
# 2 MiB per row against the per-tensor pipelined path, profiles/r02s_small_round_crossover.log.)
_SMALL_ROW_BYTES = 64 << 20
_SMALL_ROUND_BYTES = 48 << 20


def _is_small(n: int, row_bytes: int) -> bool:
    return 0 < row_bytes <= _SMALL_ROW_BYTES and n * row_bytes < _SMALL_ROUND_BYTES


class _HostRound:
    """Page-locked rows + result of the small-round path for one (device, dtype, pitch), and
    the int64 numel table of the last layout (reused while the layout repeats)."""

    def __init__(self, dtype: torch.dtype, pitch: int):
        self.dtype = dtype
        self.pitch = pitch
        self.rows = 0
        self.h_in = None
        self.h_out = torch.empty(pitch, dtype=dtype, pin_memory=True)
        self.numels_key = None
        self.numels_arr = None

    def ensure(self, n: int, numels: List[int]):
        if n > self.rows:
            self.h_in = torch.empty((n, self.pitch), dtype=self.dtype, pin_memory=True)
            self.rows = n
        key = tuple(numels)
        if key != self.numels_key:
            self.numels_arr = (ctypes.c_int64 * len(numels))(*numels)
            self.numels_key = key


_host_rounds: Dict[Tuple[torch.device, torch.dtype, int], _HostRound] = {}


def _host_round(device: torch.device, dtype: torch.dtype, pitch: int, n: int, numels: List[int]) -> _HostRound:
    """The page-locked buffers for a small round (caller holds _staging_lock)."""
    key = (device, dtype, pitch)
    hr = _host_rounds.get(key)
    if hr is None:
        hr = _host_rounds[key] = _HostRound(dtype, pitch)
    hr.ensure(n, numels)
    return hr


def _reduce_host_small(device, dtype, center: List[torch.Tensor], peers: List[List[torch.Tensor]], weights,
                       numels: List[int], total: int, pitch: int):
    """A small round through dla_host_round_* into the (contiguous) result tensors."""
    code = _wsum.dtype_code(dtype)
    with _staging_lock:
        hr = _host_round(device, dtype, pitch, len(peers), numels)
        stream = torch.cuda.current_stream(device).cuda_stream
        _lib.host_round_start(code, len(peers), [p.data_ptr() for pl in peers for p in pl], hr.numels_arr, weights,
                              hr.h_in.data_ptr(), pitch, hr.h_out.data_ptr(), stream)
        _lib.host_round_finish(code, hr.numels_arr, hr.h_out.data_ptr(), [c.data_ptr() for c in center], stream)


# list(m.parameters()) for module trees whose classes all keep nn.Module's own walk: the same order and
# the same de-duplication (pre-order over modules, a module or parameter seen before is skipped), without
# named_modules' prefix strings and generator frames — the walk over every parameter of every model is
# the host path's largest Python cost (128 google_speech ResNet-34 models: 14 080 parameters).
_WALK_METHODS = ("parameters", "named_parameters", "named_modules", "_named_members", "modules", "buffers",
                 "named_buffers")
_plain_walk_cls: Dict[type, bool] = {}


_PLAIN_SET: set = set()  # the plain classes, as the walk extension takes them


def _plain_walk(cls: type) -> bool:
    ok = _plain_walk_cls.get(cls)
    if ok is None:
        ok = all(getattr(cls, name, None) is getattr(nn.Module, name) for name in _WALK_METHODS)
        _plain_walk_cls[cls] = ok
        if ok:
            _PLAIN_SET.add(cls)
    return ok


def _native_layout(models: List[nn.Module], device: int, tensor_major: bool, ref: "nn.Module | None" = None):
    """The walk extension's one-pass layout (csrc/walk.cpp; ~10x faster per parameter than the Python
    walk): (dtype, numels, pointer table bytearray, device index), or None when the extension is not
    loaded or the round does not qualify.  Classes it has not seen are classified (models[0]'s tree)
    and the walk retried once."""
    mod = _lib.walk_module()
    if mod is None:
        return None
    r = mod.layout(models, device, _PLAIN_SET, tensor_major, ref)
    if r is None:
        fresh = [type(sub) for sub in (models[0] if ref is None else ref).modules() if type(sub) not in _plain_walk_cls]
        if any([_plain_walk(cls) for cls in fresh]):
            r = mod.layout(models, device, _PLAIN_SET, tensor_major, ref)
    if r is None:
        return None
    name, numels, table, dev = r
    return getattr(torch, name), numels, table, dev


def _parameters(model: nn.Module) -> List[nn.Parameter]:
    out: List[nn.Parameter] = []
    seen_p, seen_m = set(), set()

    def walk(mod) -> bool:
        if id(mod) in seen_m:
            return True
        if not _plain_walk(type(mod)):
            return False
        seen_m.add(id(mod))
        for p in mod._parameters.values():
            if p is not None and id(p) not in seen_p:
                seen_p.add(id(p))
                out.append(p)
        for child in mod._modules.values():
            if child is not None and not walk(child):
                return False
        return True

    return out if walk(model) else list(model.parameters())


def _host_layout(models: List[nn.Module]):
    """(dtype, numels, pointers) of a round whose models all have models[0]'s parameter shapes, one
    supported dtype and contiguous CPU storage — the models at every reference call site — with the
    parameters' host pointers peer-major, gathered in one pass without a tensor view per parameter
    (a round of 128 ResNet-34 models has 14 080 parameters: a detach + reshape + slice of each costs
    more than the GPU work); None when the round does not qualify (the general path handles it).
    The pointers come back as a ctypes array; the walk runs in the walk extension when it is loaded."""
    if not torch.cuda.is_available():
        return None
    nat = _native_layout(models, -1, tensor_major=False)
    if nat is not None:
        dtype, numels, table, _ = nat
        return dtype, numels, (ctypes.c_void_p * (len(table) // 8)).from_buffer(table)
    p0 = _parameters(models[0])
    if not p0:
        return None
    dtype = p0[0].dtype
    if dtype not in _wsum.SUPPORTED_DTYPES:
        return None
    shapes = [p.shape for p in p0]
    n_t = len(shapes)
    ptrs = []
    add = ptrs.append
    for m in models:
        ps = p0 if m is models[0] else _parameters(m)
        if len(ps) != n_t:
            return None
        for p, shape in zip(ps, shapes):
            if p.shape != shape or p.dtype is not dtype or not p.is_cpu or not p.is_contiguous():
                return None
            add(p.data_ptr())
    return dtype, [p.numel() for p in p0], (ctypes.c_void_p * len(ptrs))(*ptrs)


def _device_layout(models: List[nn.Module], ref: "nn.Module | None" = None):
    """(dtype, device, numels, tensor-major pointer table) of a round whose models all have models[0]'s
    (or `ref`'s, when given: a model outside the list) parameter shapes, one supported dtype and
    contiguous storage on ONE HIP device (models trained on the GPU, the simulator's device-resident
    averages), gathered in one pass; None otherwise (the general path handles it).  The table is
    [n_tensors x n_peers] uint64 over the listed models, as dla_wsum_multi takes it."""
    import numpy as np

    nat = _native_layout(models, -2, tensor_major=True, ref=ref)
    if nat is not None:
        dtype, numels, table, dev = nat
        return (dtype, torch.device("cuda", dev), numels,
                np.frombuffer(table, dtype=np.uint64).reshape(len(numels), len(models)))
    if ref is not None:
        models = [ref] + list(models)
    p0 = _parameters(models[0])
    if not p0 or not p0[0].is_cuda:
        return None
    dtype = p0[0].dtype
    if dtype not in _wsum.SUPPORTED_DTYPES:
        return None
    dev = p0[0].get_device()
    shapes = [p.shape for p in p0]
    n_t = len(shapes)
    rows = []
    for m in models:
        ps = p0 if m is models[0] else _parameters(m)
        if len(ps) != n_t:
            return None
        row = []
        add = row.append
        for p, shape in zip(ps, shapes):
            if p.shape != shape or p.dtype is not dtype or p.get_device() != dev or not p.is_contiguous():
                return None
            add(p.data_ptr())
        rows.append(row)
    if ref is not None:
        rows = rows[1:]
    table = np.ascontiguousarray(np.array(rows, dtype=np.uint64).T)
    return dtype, torch.device("cuda", dev), [p.numel() for p in p0], table


_flat_plans: Dict[tuple, tuple] = {}


def _flat_plan(dtype, numels: List[int]):
    """(element offsets, total elements, byte offsets as uint64, numels as a ctypes int64 array) of one
    allocation holding a layout's tensors each 256-byte aligned, cached per (dtype, layout): a device
    round of one architecture computes it once, not every round."""
    key = (dtype, tuple(numels))
    plan = _flat_plans.get(key)
    if plan is None:
        import numpy as np

        esize = torch.empty((), dtype=dtype).element_size()
        align = _ALIGN_BYTES // esize
        offs, total = [], 0
        for n_ in numels:
            offs.append(total)
            total += _round_up(max(n_, 1), align)
        if len(_flat_plans) > 64:
            _flat_plans.clear()
        plan = _flat_plans[key] = (offs, total, np.array(offs, dtype=np.uint64) * np.uint64(esize),
                                   (ctypes.c_int64 * len(numels))(*numels))
    return plan


def _device_round(models: List[nn.Module], weights, layout) -> "nn.Module | None":
    """The whole aggregate for device-resident models of one layout: deepcopy(models[0]) with fresh
    parameters (fedavg.py:20), then every parameter of every model folded straight into them by
    dla_wsum_multi(_table) from one pointer table — one launch per 128-peer pass for rounds of many
    peers, whatever the tensor count (fedavg.py:23-25).  Stream-ordered like any torch op.

    The host work around the launch is batched (a 16-model ResNet-34 round spent 2 ms
    of Python around a 0.13 ms reduce): the result's parameters are made natively, their blocks before
    the launch and their Parameter objects while the reduce runs (walk.cpp param_blocks / param_wrap: one
    caching-allocator tensor each, as deepcopy makes them, so record_stream and CUDA IPC work on the
    result — round 6; rounds 4-5 made them parts of one allocation the allocator did not know);
    models[0]'s device buffers are copied by one fused copy per dtype instead
    of one deepcopy dispatch per buffer; the module tree is cloned while the kernel runs."""
    dtype, device, numels, table = layout
    mod = _lib.walk_module()
    if mod is None or not hasattr(mod, "param_blocks"):
        return _device_round_per_tensor(models, weights, layout)
    objs = mod.tensors(models[0], _PLAIN_SET)
    if objs is None or len(objs[0]) != len(numels) or any(type(p) is not nn.Parameter for p in objs[0]):
        return _device_round_per_tensor(models, weights, layout)
    p0, b0 = objs
    nums = _flat_plan(dtype, numels)[3]
    memo = {}
    blocks, out_ptrs = mod.param_blocks(p0)
    outs = (ctypes.c_void_p * len(numels)).from_buffer(out_ptrs)
    ptrs = (ctypes.c_void_p * table.size).from_buffer(table)
    _wsum.wsum_multi_ptrs(dtype, ptrs, outs, nums, weights, device, total_elems=sum(numels))
    # while the reduce runs: the parameters' Python objects, models[0]'s buffers, the module tree
    mod.param_wrap(blocks, p0, memo)
    _seed_buffers(b0, memo)
    return _clone_value(models[0], memo)


# Device rounds of at least _GROUP_MIN models are walked and launched group by group
# (_device_round_grouped): the walk sees every parameter object once (~20 ns each: ~0.25 ms for 128
# google_speech ResNet-34 models), so one launch after the whole walk leaves the GPU idle that long.  The
# first group is small, so the GPU starts early; each later group is _DEVICE_GROUP_GROWTH times the one
# before it (a model takes ~2 us to walk and ~7 us to fold, so the next group is walked while the GPU
# folds the current one), and a tail smaller than the group due joins the last group.  Few groups keep
# the extra pass over the running sum each later group makes (dla_wsum_multi_table_acc) cheap.
_DEVICE_GROUP_FIRST = 16
_DEVICE_GROUP_GROWTH = 3
_GROUP_MIN_DEFAULT = _GROUP_MIN = 64


def _group_bounds(n: int) -> List[tuple]:
    """[(begin, end)] of the groups a device round of n models is launched in: _DEVICE_GROUP_FIRST
    models, then _DEVICE_GROUP_GROWTH times as many each group, the last group taking a tail shorter
    than its due size."""
    out, a, g = [], 0, _DEVICE_GROUP_FIRST
    while a < n:
        b = n if n - a - g < g else a + g
        out.append((a, b))
        a, g = b, g * _DEVICE_GROUP_GROWTH
    return out


def _device_round_grouped(models: List[nn.Module], weights) -> "nn.Module | None":
    """_device_round for a round of many device-resident models, launched group by group
    (_group_bounds): each group is walked (its own pointer table) and its fold launched at once, the
    groups after the first continuing the fold in the result (dla_wsum_multi_table_acc) — list order
    and the rounding of every step unchanged, so the same bits as one launch over all models
    (fedavg.py:23-25).  None when the walk extension is absent or any group does not share
    models[0]'s layout (dtype, device, shapes); the general path then handles the round."""
    mod = _lib.walk_module()
    bounds = _group_bounds(len(models))
    a0, b0_ = bounds[0]
    first = _device_layout(models[a0:b0_]) if mod is not None else None
    if first is None:
        return None
    dtype, device, numels, table = first
    # models[0]'s own objects and the result's fresh parameter blocks (walk.cpp param_blocks), before the
    # first launch writes into them; their Parameter objects while it runs (param_wrap)
    objs = mod.tensors(models[0], _PLAIN_SET) if hasattr(mod, "param_blocks") else None
    if objs is None or len(objs[0]) != len(numels) or any(type(p) is not nn.Parameter for p in objs[0]):
        return None
    p0, b0 = objs
    nums = _flat_plan(dtype, numels)[3]
    memo = {}
    blocks, out_ptrs = mod.param_blocks(p0)
    outs = (ctypes.c_void_p * len(numels)).from_buffer(out_ptrs)
    _wsum.wsum_multi_ptrs(dtype, (ctypes.c_void_p * table.size).from_buffer(table), outs, nums,
                          weights[a0:b0_], device, total_elems=sum(numels))
    mod.param_wrap(blocks, p0, memo)
    for a, b in bounds[1:]:
        # each later group checked against models[0]'s layout (shapes, dtype, device) in its own walk
        lay = _device_layout(models[a:b], ref=models[0])
        if lay is None or lay[0] is not dtype or lay[1] != device or lay[2] != numels:
            return None
        _wsum.wsum_multi_ptrs(dtype, (ctypes.c_void_p * lay[3].size).from_buffer(lay[3]), outs, nums,
                              weights[a:b], device, acc_in=True)
    _seed_buffers(b0, memo)
    return _clone_value(models[0], memo)


def _seed_buffers(buffers, memo: dict) -> None:
    """deepcopy of models[0]'s device buffers (fedavg.py:20 copies them, it does not average them) in
    one gather per (device, dtype) group: the copies are views of one fresh allocation each, seeded
    into the deepcopy memo.  Buffers that are not plain dense tensors without grad keep the stock
    deepcopy.  The walk extension does it in one native call (walk.cpp buffer_copies)."""
    mod = _lib.walk_module()
    if mod is not None:
        mod.buffer_copies(buffers, memo)
        return
    groups: Dict[tuple, list] = {}
    uses: Dict[int, int] = {}
    dense = [b for b in {id(b): b for b in buffers}.values()
             if type(b) is torch.Tensor and b.layout is torch.strided and b.device.type in ("cpu", "cuda")]
    for b in dense:
        key = b.untyped_storage().data_ptr()
        uses[key] = uses.get(key, 0) + 1
    for b in dense:
        if (not b.requires_grad and b.is_contiguous() and id(b) not in memo
                and uses[b.untyped_storage().data_ptr()] == 1):
            groups.setdefault((b.device, b.dtype), []).append(b)
    for bs in groups.values():
        if len(bs) < 2:
            continue
        flat = torch._C._nn.flatten_dense_tensors(bs)
        for b, c in zip(bs, torch._C._nn.unflatten_dense_tensors(flat, bs)):
            memo[id(b)] = c


def _device_round_per_tensor(models: List[nn.Module], weights, layout) -> "nn.Module | None":
    """_device_round for module trees the walk extension cannot read (no extension, Parameter
    subclasses): one fresh tensor per parameter, the stock deepcopy of every buffer."""
    dtype, device, numels, table = layout
    memo = _fresh_params(models[0])
    params = [memo[id(p)] for p in models[0].parameters()] if len(memo) == len(numels) else []
    if len(params) != len(numels) or not all(c.is_contiguous() and c.device == device for c in params):
        return None
    ptrs = (ctypes.c_void_p * table.size).from_buffer(table)
    outs = (ctypes.c_void_p * len(params))(*[c.data_ptr() for c in params])
    nums = (ctypes.c_int64 * len(numels))(*numels)
    _wsum.wsum_multi_ptrs(dtype, ptrs, outs, nums, weights, device, total_elems=sum(numels))
    return _clone_value(models[0], memo)


def _small_round(models: List[nn.Module], weights, layout) -> "nn.Module | None":
    """The whole aggregate for a small round of same-layout, one-dtype, contiguous CPU
    models (the reference's call sites: GL merges N=2 every round): one native call packs
    every peer into page-locked rows and enqueues the reduce, which reads the rows and writes
    the page-locked result across PCIe (no staging DMA, dla_host_round_start); the result
    module is built on the host while it runs, then one call waits and unpacks into its
    parameters (dla_host_round_finish).  None when the round is not small."""
    dtype, numels, ptrs = layout
    total = sum(numels)
    esize = torch.empty((), dtype=dtype).element_size()
    n = len(models)
    if not _is_small(n, total * esize):
        return None
    device = _wsum.require_device(None)
    pitch = _round_up(total, _ALIGN_BYTES // esize)
    code = _wsum.dtype_code(dtype)
    with _staging_lock:
        hr = _host_round(device, dtype, pitch, n, numels)
        stream = torch.cuda.current_stream(device).cuda_stream
        _lib.host_round_start(code, n, ptrs, hr.numels_arr, weights, hr.h_in.data_ptr(), pitch, hr.h_out.data_ptr(),
                              stream)
        # the kernel now reads hr.h_in / writes hr.h_out across PCIe: every way out of this block
        # waits for it, so the next round cannot repack those rows under a running kernel
        try:
            center = _center_copy(models[0])  # overlaps the reduce
            params = list(center.parameters())
            ok = len(params) == len(numels) and all(c.is_contiguous() for c in params)
        except BaseException:
            torch.cuda.current_stream(device).synchronize()
            raise
        if not ok:
            torch.cuda.current_stream(device).synchronize()
            return None
        _lib.host_round_finish(code, hr.numels_arr, hr.h_out.data_ptr(), [c.data_ptr() for c in params], stream)
    return center


def _large_round(models: List[nn.Module], weights, layout) -> "nn.Module | None":
    """A large round of same-layout CPU models through dla_host_reduce_launch from the pointer table
    of _host_layout: every GPU of the host path (_devices_for) streams its parameter bucket in packed
    chunks (one DMA per chunk) on a library thread of its own; the averaged elements land in the
    result's parameters.  None when the result's parameters are not dense CPU tensors."""

    from accdfl_amd.core.sharding import bucket_bounds

    dtype, numels, ptrs = layout
    n = len(models)
    esize = torch.empty((), dtype=dtype).element_size()
    total = sum(numels)
    align = _ALIGN_BYTES // esize
    device = _wsum.require_device(None)
    devices = _devices_for(device, total * esize)
    devices = devices[:max(1, min(len(devices), (total * esize) // _MIN_SHARD_BYTES))]
    # Every GPU bucket starts streaming through its GPU at once, on a thread of the library's own
    # (dla_host_reduce_launch: no interpreter lock needed while it runs); this thread allocates the
    # result's parameters meanwhile, publishes them (out_arr, then ready = 1: only the native first
    # unpack waits for them), then clones the module tree around them (deepcopy of models[0],
    # fedavg.py:20) while the round streams on, and joins.
    code = _wsum.dtype_code(dtype)
    tensor_arr = ptrs  # a ctypes array (_host_layout)
    numel_arr = (ctypes.c_int64 * len(numels))(*numels)
    out_arr = (ctypes.c_void_p * len(numels))()
    ready = ctypes.c_int(0)
    with _staging_lock:
        launched = []
        center = None
        try:
            for i, (dev, (s, e)) in enumerate(zip(devices, bucket_bounds(total, len(devices), align))):
                if s >= e:
                    continue
                chunk = _native_chunk(n, esize, e - s, align)
                st = _get_native_staging(dev, dtype, i if len(devices) > 1 else -1, n, chunk)
                compute = torch.cuda.current_stream(dev)
                st.copy_stream.wait_stream(compute)  # earlier users of the device staging are done
                launched.append(_lib.host_reduce_launch(
                    dev.index, code, n, tensor_arr, numel_arr, weights, out_arr, ready, s, e, chunk,
                    st.h_stage.data_ptr(), st.d_stage.data_ptr(), st.h_out.data_ptr(), st.d_out.data_ptr(),
                    compute.cuda_stream, st.copy_stream.cuda_stream))
            memo = _fresh_params(models[0])
            params = [memo.get(id(p)) for p in models[0].parameters()] if len(memo) == len(numels) else []
            if len(params) == len(numels) and all(c is not None and c.is_cpu and c.is_contiguous() for c in params):
                for i, c in enumerate(params):
                    out_arr[i] = c.data_ptr()
                ready.value = 1
                center = _clone_value(models[0], memo)
        finally:
            if ready.value == 0:
                ready.value = -1  # no result tensors: the native calls drain and give up
            errors = []
            for job in launched:  # every bucket has finished with the staging before the lock goes
                try:
                    job.join()
                except _lib.DlaggError as err:
                    errors.append(err)
        if ready.value < 0:
            return None  # the general path handles this round (the abandoned calls' errors are expected)
        if errors:
            raise errors[0]
    return center


def _stage_rows(st, dev, k: int, flat: List[torch.Tensor], numels: List[int], s: int, e: int):
    """Peer k's elements [s, e) -> row k of st.d_in (pinned pack + async H2D on the copy stream)."""
    parts = _flat_slices(flat, numels, s, e)
    if all(t.device.type == "cpu" for t in flat):
        row = st.h_in[k, : e - s]
        if len(parts) == 1:
            row.copy_(parts[0])
        else:
            torch.cat(parts, out=row)
        with torch.cuda.device(dev), torch.cuda.stream(st.copy_stream):
            st.d_in[k, : e - s].copy_(row, non_blocking=True)
    else:
        with torch.cuda.device(dev), torch.cuda.stream(st.copy_stream):
            torch.cat([t.to(dev, non_blocking=True) for t in parts], out=st.d_in[k, : e - s])


def _reduce_rows(st, dev, weights, center: List[torch.Tensor], numels: List[int], s: int, e: int, h_out):
    """Reduce rows 0..n-1 of st.d_in after the copies land, then D2H the bucket [s, e)
    straight into the result's parameters (h_out is None) or into h_out[s:e]."""
    compute = torch.cuda.current_stream(dev)
    compute.wait_stream(st.copy_stream)
    with torch.cuda.device(dev):
        _wsum.wsum_rows(st.d_in, weights, e - s, out=st.d_out)
        dst = _flat_slices(center, numels, s, e) if h_out is None else [h_out[s:e]]
        off = 0
        for d in dst:
            d.copy_(st.d_out[off:off + d.numel()], non_blocking=True)
            off += d.numel()


_PIPE_CHUNKS = 4               # element chunks per bucket in the pipelined host path
_PIPE_MIN_CHUNK_BYTES = 8 << 20


def _bucket_pipelined(st, dev, flats: List[List[torch.Tensor]], numels: List[int], s: int, e: int, weights,
                      center: List[torch.Tensor], h_out, align: int):
    """Bucket [s, e) of every peer through one GPU in element chunks: chunk c's H2D copies
    go straight from the (pageable) parameters, then its reduce and its D2H are enqueued,
    so the D2H of chunk c runs while chunk c+1 is still coming in (PCIe is full duplex).
    Every element still folds all peers in list order: the result is unchanged."""
    n = len(flats)
    esize = st.d_in.element_size()
    chunk = max(_PIPE_MIN_CHUNK_BYTES // esize, -(-(e - s) // _PIPE_CHUNKS))
    chunk = _round_up(chunk, align)
    compute = torch.cuda.current_stream(dev)
    with torch.cuda.device(dev):
        for cs in range(s, e, chunk):
            ce = min(e, cs + chunk)
            with torch.cuda.stream(st.copy_stream):
                for k in range(n):
                    off = cs - s
                    for t in _flat_slices(flats[k], numels, cs, ce):
                        st.d_in[k, off:off + t.numel()].copy_(t if t.device == dev or t.device.type == "cpu"
                                                              else t.to(dev, non_blocking=True), non_blocking=True)
                        off += t.numel()
            compute.wait_stream(st.copy_stream)
            _wsum.wsum_rows(st.d_in[:, cs - s:ce - s], weights, ce - cs, out=st.d_out[cs - s:ce - s])
            dst = _flat_slices(center, numels, cs, ce) if h_out is None else [h_out[cs:ce]]
            off = cs - s
            for d in dst:
                d.view(-1).copy_(st.d_out[off:off + d.numel()], non_blocking=True)
                off += d.numel()
        compute.synchronize()


class _NativeStaging:
    """Double-buffered chunk staging of dla_host_reduce for one (device, dtype, slot): page-locked
    h_stage / h_out and device d_stage / d_out, grown on demand and reused across rounds."""

    def __init__(self, device: torch.device, dtype: torch.dtype):
        self.device = device
        self.dtype = dtype
        self.rows = self.chunk = 0
        self.h_stage = self.d_stage = self.h_out = self.d_out = None
        self.copy_stream = torch.cuda.Stream(device)

    def ensure(self, rows: int, chunk: int):
        """Room for two chunks of ``rows`` rows of ``chunk`` elements.  The staging grows with the
        byte footprint rows * chunk, not with the two maxima apart: the chunk shrinks as the peer
        count grows (_native_chunk), so a 2-peer round of a 25 M model (chunk 3.1 M) followed by a
        64-peer round (chunk 131 K) needs 2 x 8.4 M elements, not 2 x 64 x 3.1 M (1.6 GB of
        page-locked host memory plus as much HBM).  dla_host_reduce lays the rows out from the
        call's own (n_peers, chunk_elems), so any buffer of at least that size serves."""
        stage = 2 * rows * chunk
        if self.h_stage is None or self.h_stage.numel() < stage:
            self.h_stage = self.d_stage = None
            self.h_stage = torch.empty(stage, dtype=self.dtype, pin_memory=True)
            self.d_stage = torch.empty(stage, dtype=self.dtype, device=self.device)
        if self.h_out is None or self.h_out.numel() < 2 * chunk:
            self.h_out = self.d_out = None
            self.h_out = torch.empty(2 * chunk, dtype=self.dtype, pin_memory=True)
            self.d_out = torch.empty(2 * chunk, dtype=self.dtype, device=self.device)
        self.rows, self.chunk = rows, chunk


_native_staging: Dict[Tuple[torch.device, torch.dtype, int], _NativeStaging] = {}

# Bytes of every peer's rows per chunk of dla_host_reduce (two chunks in flight): large enough that
# one DMA per chunk runs at the PCIe rate, small enough that packing chunk c+1 overlaps the DMA of
# chunk c from the start of the round.
_NATIVE_CHUNK_BYTES = int(float(_lib.tuning_env("ACCDFL_AMD_HOST_CHUNK_MB", "32")) * (1 << 20))


_NATIVE_MIN_CHUNK_BYTES = 2 << 20


def _native_chunk(n: int, esize: int, bucket: int, align: int) -> int:
    """Elements per peer row of a dla_host_reduce chunk: 32 MiB of rows, but at least 8 chunks per
    bucket down to 2 MiB — nothing crosses PCIe until the first chunk is packed, so a round of one
    or two full chunks waits a whole pack before its DMA starts (2 x 4.9 M fp32: 1.58 ms in 32 MiB
    chunks against 1.48 for per-tensor DMAs, profiles/r02zk_crossover.log)."""
    target = min(_NATIVE_CHUNK_BYTES, max(_NATIVE_MIN_CHUNK_BYTES, n * bucket * esize // 8))
    chunk = max(align, target // (n * esize) // align * align)
    return min(chunk, _round_up(bucket, align))


def _get_native_staging(device: torch.device, dtype: torch.dtype, slot: int, rows: int,
                        chunk: int) -> _NativeStaging:
    """(caller holds _staging_lock)"""
    key = (device, dtype, slot)
    st = _native_staging.get(key)
    if st is None:
        st = _native_staging[key] = _NativeStaging(device, dtype)
    st.ensure(rows, chunk)
    return st


def _bucket_native(st: _NativeStaging, dev, flats: List[List[torch.Tensor]], numels: List[int], s: int, e: int,
                   weights, center: List[torch.Tensor], h_out, align: int):
    """Bucket [s, e) of every peer through one GPU by dla_host_reduce: per chunk, one threaded pack
    of every peer's slices into page-locked rows, ONE H2D DMA, the list-order reduce, the D2H and
    the unpack into the result, two chunks in flight.  (The pipelined path issues one DMA per
    tensor per peer per chunk: 14 080 per chunk for 128 ResNet-34 models.)"""
    n = len(flats)
    dtype = st.dtype
    chunk = _native_chunk(n, st.h_stage.element_size(), e - s, align)
    parts = [_flat_slices(f, numels, s, e) for f in flats]
    sizes = [t.numel() for t in parts[0]]
    ptrs = [t.data_ptr() for pl in parts for t in pl]
    # one output pointer per tensor slice, as dla_host_reduce reads them (a non-dense result lands in
    # h_out, cut at the same tensor boundaries)
    outs = _flat_slices(center if h_out is None else list(torch.split(h_out, numels)), numels, s, e)
    compute = torch.cuda.current_stream(dev)
    st.copy_stream.wait_stream(compute)  # earlier users of the device staging are done
    with torch.cuda.device(dev):
        _lib.host_reduce(_wsum.dtype_code(dtype), n, ptrs, sizes, weights, [o.data_ptr() for o in outs], 0, e - s,
                         chunk, st.h_stage.data_ptr(), st.d_stage.data_ptr(), st.h_out.data_ptr(),
                         st.d_out.data_ptr(), compute.cuda_stream, st.copy_stream.cuda_stream)


# How the host-staged path moves a large round (ACCDFL_AMD_HOST_PATH):
# * "native" (default): one host thread per GPU, each streaming its bucket through
#   dla_host_reduce (_bucket_native: threaded pack into page-locked chunk rows, one DMA per chunk);
# * "pipelined": one host thread per GPU, each streaming its bucket through _bucket_pipelined
#   (one H2D per tensor per peer per chunk, straight from the pageable parameters);
# * "packed": one thread packing every peer into pinned staging peer-major and issuing the DMAs.
# Peers that are not contiguous CPU tensors take "pipelined".
_HOST_PATHS = ("native", "pipelined", "packed")
_HOST_PATH = _lib.tuning_env("ACCDFL_AMD_HOST_PATH", "native")
if _HOST_PATH not in _HOST_PATHS:
    raise ValueError("ACCDFL_AMD_HOST_PATH must be one of %s" % (_HOST_PATHS,))


def set_host_path(mode: str) -> None:
    global _HOST_PATH
    if mode not in _HOST_PATHS:
        raise ValueError("host path must be one of %s" % (_HOST_PATHS,))
    _HOST_PATH = mode


def host_path() -> str:
    return _HOST_PATH


def set_shard_threads(enabled: bool) -> None:
    """True: one host thread per GPU (the default "native" path); False: the serial "packed" path."""
    set_host_path("native" if enabled else "packed")


def _reduce_host_staged(devices: List[torch.device], dtype, center: List[torch.Tensor],
                        peers: List[List[torch.Tensor]], weights):
    """One dtype group, every model contributing to every tensor: pack -> H2D -> reduce -> D2H,
    bucket-sharded over ``devices`` (each bucket over its own GPU's PCIe link)."""
    from accdfl_amd.core.sharding import bucket_bounds

    numels = [c.numel() for c in center]
    total = sum(numels)
    if total == 0:
        return
    esize = torch.empty((), dtype=dtype).element_size()
    align = _ALIGN_BYTES // esize
    if (_is_small(len(peers), total * esize) and all(c.is_contiguous() for c in center)
            and all(p.device.type == "cpu" and p.is_contiguous() for pl in peers for p in pl)):
        _reduce_host_small(devices[0], dtype, center, peers, weights, numels, total, _round_up(total, align))
        return
    g_max = max(1, min(len(devices), (total * esize) // _MIN_SHARD_BYTES))
    devices = devices[:g_max]
    bounds = bucket_bounds(total, len(devices), align)
    n = len(peers)
    flats = [[p.detach().reshape(-1) for p in pl] for pl in peers]
    native = _HOST_PATH == "native" and all(t.device.type == "cpu" and t.is_contiguous() for f in flats for t in f)
    with _staging_lock:
        stages = []
        for dev, (s, e) in zip(devices, bounds):
            if native:
                st = _get_native_staging(dev, dtype, len(stages) if len(devices) > 1 else -1, n,
                                         _native_chunk(n, esize, max(e - s, 1), align))
            else:
                st = _get_staging(dev, dtype) if len(devices) == 1 else _get_staging_sharded(dev, dtype, len(stages))
                st.ensure(n, _round_up(max(e - s, 1), align))
                st.copy_stream.wait_stream(torch.cuda.current_stream(dev))  # previous users of d_in are done
            stages.append(st)
        # D2H straight into the result's parameters when they are dense (pageable ones through the
        # runtime's staging, page-locked ones directly); non-dense results go through one pinned buffer.
        direct = all(c.is_contiguous() for c in center)
        h_out = None if direct else torch.empty(total, dtype=dtype, pin_memory=True)
        jobs = [(st, dev, s, e) for st, dev, (s, e) in zip(stages, devices, bounds) if s < e]
        _run_bucket_jobs(jobs, devices, flats, numels, weights, center, h_out, align, n)
        if not direct:
            for c, o in zip(center, torch.split(h_out, numels)):
                c.copy_(o.view_as(c))


def _run_bucket_jobs(jobs, devices, flats, numels, weights, center, h_out, align, n):
    """Every bucket's H2D -> reduce -> D2H, one thread per GPU (pipelined) or peer-major from
    this thread (packed); returns when every D2H has landed."""
    if _HOST_PATH != "packed":
        from concurrent.futures import ThreadPoolExecutor

        def bucket(job):
            st, dev, s, e = job
            with torch.no_grad():  # grad mode is per thread; the result's parameters are leaves
                if isinstance(st, _NativeStaging):
                    _bucket_native(st, dev, flats, numels, s, e, weights, center, h_out, align)
                else:
                    _bucket_pipelined(st, dev, flats, numels, s, e, weights, center, h_out, align)

        if len(jobs) == 1:
            bucket(jobs[0])
        else:
            with ThreadPoolExecutor(max_workers=len(jobs)) as pool:
                list(pool.map(bucket, jobs))  # re-raises the first failure
    else:
        for k in range(n):  # peer-major: every GPU's DMA starts as early as possible
            for st, dev, s, e in jobs:
                _stage_rows(st, dev, k, flats[k], numels, s, e)
        for st, dev, s, e in jobs:
            _reduce_rows(st, dev, weights, center, numels, s, e, h_out)
        for dev in devices:
            torch.cuda.current_stream(dev).synchronize()


def _reduce_device_resident(dtype, center: List[torch.Tensor], peers: List[List[torch.Tensor]], weights):
    """One dtype group, all tensors on the device: reduce straight into the center params."""
    outs, tmp = [], []
    for i, c in enumerate(center):
        if c.is_contiguous():
            outs.append(c)
        else:
            t = torch.empty(c.shape, dtype=c.dtype, device=c.device)
            outs.append(t)
            tmp.append((c, t))
    _wsum.wsum_multi([[p.detach() if p.is_contiguous() else p.detach().contiguous() for p in pl] for pl in peers],
                     weights, outs)
    for c, t in tmp:
        c.copy_(t)


def _reduce_multi_device(center: List[torch.Tensor], peers: List[List[torch.Tensor]], weights,
                         devices: "List[torch.device] | None" = None):
    """One dtype group, every tensor on a GPU but not all on one (e.g. models trained on
    different GPUs of the aggregating node): each parameter is reduced in place of the
    result's tensor by dla_wsum_sharded, its buckets spread over the GPUs holding the peers
    (the result's GPU first) and each bucket read over xGMI where it lives elsewhere — no
    staging copy of any peer.  Parameters under 8 MB per GPU use fewer buckets (one: a single
    reduce on the result's GPU).  ``devices`` overrides the bucket placement (tests)."""
    for i, c in enumerate(center):
        terms = [pl[i].detach() if pl[i].is_contiguous() else pl[i].detach().contiguous() for pl in peers]
        if devices is None:
            others = sorted({t.device.index for t in terms} - {c.device.index})
            devs = [c.device] + [torch.device("cuda", d) for d in others]
        else:
            devs = list(devices)
        g = max(1, min(len(devs), c.numel() * c.element_size() // _MIN_SHARD_BYTES))
        out = c if c.is_contiguous() else torch.empty(c.shape, dtype=c.dtype, device=c.device)
        _wsum.wsum_sharded([t.reshape(-1) for t in terms], weights, devs[:g] if devices is None else devs,
                           out=out.view(-1))
        if out is not c:
            c.copy_(out)


def _reduce_param(device, center: torch.Tensor, terms: List[torch.Tensor], weights: List[float]):
    """A single parameter with its own contributor set (zip truncation)."""
    dev_terms = [t.detach().to(device).contiguous() for t in terms]
    out = _wsum.wsum(dev_terms, weights)
    center.copy_(out.view_as(center))
    if center.device.type == "cpu":
        torch.cuda.current_stream(device).synchronize()


def _reduce_param_mixed(device, center: torch.Tensor, terms: List[torch.Tensor], weights: List[float]):
    """A parameter whose contributors do not share models[0]'s dtype (dla_wsum_mixed: products
    rounded in each peer's dtype, sums in the centre's after promotion, fedavg.py:25)."""
    if center.numel() == 0:
        return
    dev_terms = [t.detach().to(device).contiguous() for t in terms]
    out = torch.empty(center.numel(), dtype=center.dtype, device=device)
    _wsum.wsum_mixed([t.view(-1) for t in dev_terms], weights, out)
    center.copy_(out.view_as(center))
    if center.device.type == "cpu":
        torch.cuda.current_stream(device).synchronize()


def reduce_parameters(center_params: List[torch.Tensor], peer_params: List[List[torch.Tensor]],
                      weights: List[float]) -> None:
    """fedavg.py:21-25 on parameter lists: center_params[i] <- FedAvg over the models
    that have an i-th parameter.  ``center_params`` is a deepcopy of models[0]'s.  Parameters whose
    contributors have other dtypes than models[0]'s are folded with the reference's promotion
    (_reduce_param_mixed); a shape mismatch raises (the reference would broadcast)."""
    n = len(peer_params)
    if not center_params:
        return
    first = center_params[0].device
    device = _wsum.require_device(first if first.type == "cuda" else None)
    full: Dict[torch.dtype, List[int]] = {}
    partial: List[int] = []
    mixed: List[int] = []
    for i, c in enumerate(center_params):
        _wsum.dtype_code(c.dtype)
        ks = [k for k in range(n) if len(peer_params[k]) > i]
        same = True
        for k in ks:
            p = peer_params[k][i]
            if p.shape != c.shape:
                raise RuntimeError("FedAvg: parameter %d of model %d has shape %s, model 0 has %s"
                                   % (i, k, tuple(p.shape), tuple(c.shape)))
            if p.dtype != c.dtype:
                _wsum.dtype_code(p.dtype)
                same = False
        if not same:
            mixed.append(i)
        elif len(ks) == n:
            full.setdefault(c.dtype, []).append(i)
        else:
            partial.append(i)
    for i in mixed:
        ks = [k for k in range(n) if len(peer_params[k]) > i]
        _reduce_param_mixed(device, center_params[i], [peer_params[k][i] for k in ks], [weights[k] for k in ks])
    for dtype, idx in full.items():
        center = [center_params[i] for i in idx]
        peers = [[peer_params[k][i] for i in idx] for k in range(n)]
        resident = all(t.device == device for t in center) and all(t.device == device for pl in peers for t in pl)
        if resident:
            _reduce_device_resident(dtype, center, peers, weights)
        elif all(t.device.type == "cuda" for t in center) and all(t.device.type == "cuda" for pl in peers for t in pl):
            _reduce_multi_device(center, peers, weights)
        else:
            round_bytes = n * sum(c.numel() for c in center) * center[0].element_size()
            _reduce_host_staged(_devices_for(device, round_bytes), dtype, center, peers, weights)
    for i in partial:
        ks = [k for k in range(n) if len(peer_params[k]) > i]
        _reduce_param(device, center_params[i], [peer_params[k][i] for k in ks], [weights[k] for k in ks])


# copy.deepcopy's own protocol for an nn.Module (copy._reconstruct): y = cls.__new__(cls),
# state = deepcopy(x.__getstate__()), y.__setstate__(state).  _clone_value restates it for module
# classes that keep torch's __getstate__ and have no other copy hook, and for the plain dicts,
# OrderedDicts and empty sets a module's __dict__ holds; everything else (tensors, buffers,
# lists, user objects, classes with their own protocol) goes through copy.deepcopy with the same
# memo, so identity (tied weights, shared submodules) is preserved exactly as deepcopy does.
_ATOMIC = frozenset({type(None), bool, int, float, complex, str, bytes, torch.dtype, torch.device})
_plain_module_cls: Dict[type, bool] = {}
_PLAIN_MODULE_SET: set = set()  # the classes _plain_module accepts, as the walk extension takes them
# the tree cloned by the walk extension (walk.cpp clone_value: the same order and memo, no Python call
# per seeded entry, dict, container or plain module)
_NATIVE_CLONE = True


def _setstate_full_state():
    """The attribute names of a fresh nn.Module when this torch's nn.Module.__setstate__, given a state
    holding all of them, only copies it into the module's __dict__ (its other lines add attributes old
    checkpoints lack); the walk extension then sets such a state as the clone's __dict__ without calling
    it.  None (always call it) when this torch's function does anything else with a full state."""
    m = nn.Module()
    state = {k: v for k, v in m.__dict__.items() if k != "_compiled_call_impl"}
    y = nn.Module.__new__(nn.Module)
    try:
        nn.Module.__setstate__(y, dict(state))
    except Exception:  # noqa: BLE001 — any other behaviour: keep the call
        return None
    d = y.__dict__
    if list(d) != list(state) or any(d[k] is not v for k, v in state.items()):
        return None
    return tuple(state)


_SETSTATE_FN = nn.Module.__dict__["__setstate__"]
_FULL_STATE = _setstate_full_state()
_SETSTATE_ARGS = (_SETSTATE_FN, _FULL_STATE) if _FULL_STATE is not None else (None, None)


def _plain_module(cls: type) -> bool:
    ok = _plain_module_cls.get(cls)
    if ok is None:
        ok = (issubclass(cls, nn.Module) and cls.__getstate__ is nn.Module.__getstate__
              and cls.__reduce_ex__ is object.__reduce_ex__ and cls.__reduce__ is object.__reduce__
              and getattr(cls, "__deepcopy__", None) is None and cls not in copyreg.dispatch_table
              and not any("__slots__" in c.__dict__ for c in cls.__mro__))
        _plain_module_cls[cls] = ok
        if ok:
            _PLAIN_MODULE_SET.add(cls)
    return ok


def _clone_fallback(v, memo: dict):
    """The walk extension's fallback for an object its clone does not take itself: a module class not
    yet classified (classified now, then cloned natively), else copy.deepcopy with the same memo."""
    if _plain_module(type(v)):
        return _lib.walk_module().clone_value(v, memo, _ATOMIC, _PLAIN_MODULE_SET, _clone_fallback, OrderedDict,
                                              *_SETSTATE_ARGS)
    return copy.deepcopy(v, memo)


def _clone_value(v, memo: dict):
    mod = _lib.walk_module() if _NATIVE_CLONE else None
    if mod is not None:
        return mod.clone_value(v, memo, _ATOMIC, _PLAIN_MODULE_SET, _clone_fallback, OrderedDict, *_SETSTATE_ARGS)
    t = type(v)
    if t in _ATOMIC:
        return v
    y = memo.get(id(v), memo)
    if y is not memo:
        return y
    if t is dict or t is OrderedDict:
        y = t()
        memo[id(v)] = y
        get = memo.get
        for k, x in v.items():
            c = get(id(x), memo)  # seeded entries (parameters, buffers) without a call each
            y[k if type(k) in _ATOMIC else copy.deepcopy(k, memo)] = c if c is not memo else _clone_value(x, memo)
        return y
    if t is set and not v:
        y = set()
        memo[id(v)] = y
        return y
    if _plain_module(t):
        y = t.__new__(t)
        memo[id(v)] = y
        state = {k: _clone_value(x, memo) for k, x in v.__dict__.items() if k != "_compiled_call_impl"}
        y.__setstate__(state)
        return y
    return copy.deepcopy(v, memo)


def _center_copy(model0: nn.Module, large: bool = True) -> nn.Module:
    """``copy.deepcopy(models[0])`` (fedavg.py:20) whose parameters are fresh,
    uninitialised tensors of the same shape, strides, dtype, device and
    ``requires_grad``: the reduce overwrites every one of them, so copying models[0]'s
    values first (and page-faulting P fresh elements: 16 ms of a 35 ms host-inclusive
    8 x 25 M reduce) is wasted.  Contiguous CPU parameters come from
    core/host_memory.result_tensor (tensors of 1 MiB and more: pre-faulted pooled pageable memory
    by default — a fresh 19.7 MB result costs 1.65 ms of page faults, as much as the PCIe transfer
    of a 2-model ResNet-8 round; ``large=False`` allocates every parameter fresh).
    Buffers and every other attribute are deep-copied exactly as in the reference (the module
    tree through _clone_value, deepcopy's protocol without its per-object dispatch: the GL
    merge of two GNLeNet models builds this copy every round); the buffers of each (device, dtype) are
    copied by one gather into one fresh allocation (_seed_buffers) instead of a deepcopy each."""
    mod = _lib.walk_module()
    objs = mod.tensors(model0, _PLAIN_SET) if mod is not None else None
    memo = _flat_params(mod, objs[0], large) if objs is not None else None
    if memo is None:
        memo = _fresh_params(model0, large)
    if objs is not None and len(objs[1]) > 1:
        _seed_buffers(objs[1], memo)
    return _clone_value(model0, memo)


def _flat_params(mod, params: list, large: bool) -> "dict | None":
    """_fresh_params for contiguous CPU nn.Parameters of one dtype, in one allocation: the deepcopy memo
    id(parameter) -> an nn.Parameter over its own 256-byte-aligned part of one fresh tensor (each with a
    storage of its own, walk.cpp alias_of: pickles like a deepcopied tensor), made natively — a GL merge
    builds this copy every round.  The allocation is pooled pre-faulted memory when large (as
    _fresh_params gives each large parameter).  None when the parameters do not qualify."""
    if not params:
        return None
    dtype = params[0].dtype
    for p in params:
        if type(p) is not nn.Parameter or p.dtype is not dtype or not p.is_cpu or not p.is_contiguous():
            return None
    offs, total, _, _ = _flat_plan(dtype, [p.numel() for p in params])
    flat = (_host_memory.result_tensor((total,), dtype) if large
            else torch.empty(total, dtype=dtype))
    memo = {}
    mod.param_views(flat, params, offs, memo)
    return memo


def _fresh_params(model0: nn.Module, large: bool = True) -> dict:
    """The deepcopy memo _center_copy seeds: id(parameter) -> a fresh, uninitialised nn.Parameter of
    the same shape, strides, dtype, device and requires_grad (nn.Parameter subclasses are left to
    the stock deepcopy)."""
    memo = {}
    for p in model0.parameters():
        if id(p) in memo or type(p) is not nn.Parameter:
            continue  # Parameter subclasses keep the stock deepcopy
        if p.device.type == "cpu":
            if large and p.is_contiguous() and p.numel() * p.element_size() >= _host_memory.POOL_MIN_BYTES:
                data = _host_memory.result_tensor(p.shape, p.dtype)
            else:
                data = torch.empty_strided(p.size(), p.stride(), dtype=p.dtype)
        else:
            data = torch.empty_strided(p.size(), p.stride(), dtype=p.dtype, device=p.device)
        memo[id(p)] = nn.Parameter(data, p.requires_grad)
    return memo


class FedAvg(GradientAggregation):

    @staticmethod
    def aggregate(models: List[nn.Module], weights: List[float]):
        if not weights:
            weights = [float(1. / len(models)) for _ in range(len(models))]
        else:
            assert len(weights) == len(models)

        with torch.no_grad():
            if len(models) > 0:
                # models already on a GPU skip the host-layout attempt (a failed walk of every model)
                p_first = next(iter(models[0].parameters()), None)
                layout = _host_layout(models) if p_first is None or not p_first.is_cuda else None
                if layout is not None:
                    done = _small_round(models, list(weights), layout)
                    if done is None and _HOST_PATH == "native":
                        done = _large_round(models, list(weights), layout)
                    if done is not None:
                        return done
                else:
                    if len(models) >= _GROUP_MIN and p_first is not None and p_first.is_cuda:
                        done = _device_round_grouped(models, list(weights))
                        if done is not None:
                            return done
                    dev_layout = _device_layout(models)
                    if dev_layout is not None:
                        done = _device_round(models, list(weights), dev_layout)
                        if done is not None:
                            return done
            center_model = _center_copy(models[0])
            reduce_parameters(list(center_model.parameters()), [list(m.parameters()) for m in models],
                              list(weights))
            return center_model
