"""Host memory of the averaged model's CPU parameters.

The reference returns ``deepcopy(models[0])`` with ordinary (pageable) CPU tensors
(accdfl/core/gradient_aggregation/fedavg.py:20), and callers keep that model: the simulator
holds one per node.  The reduce's D2H has to land in those tensors, and on the MI355X hosts
measured the cost of a fresh pageable result is not the copy but faulting its pages in: a
100 MB D2H takes 1.8 ms into pageable memory already touched, 11.2 ms into fresh memory,
and 1.8 ms into page-locked memory (profiles/r02f_result_memory.log).  Three modes, chosen
by ``ACCDFL_AMD_RESULT_MEMORY`` or ``set_result_memory``:

* ``pooled`` (default): the large result tensors (>= 1 MiB) are ordinary pageable memory
  taken from a pool of already-faulted blocks (anonymous mmaps, transparent huge pages
  requested).  A block returns to the pool when the last tensor using it is freed, and the
  pool keeps at most ``POOL_FREE_BYTES`` of free blocks.  Nothing is page-locked.
* ``pinned``: the result tensors of >= 1 MiB are allocated page-locked
  (``is_pinned()``).  As fast, but they stay page-locked for the model's lifetime and
  torch's caching host allocator keeps freed blocks page-locked too, so page-locked host
  memory grows with the number of results kept.
* ``pageable``: fresh pageable tensors (``torch.empty``), every page faulted in by the D2H.
"""
from __future__ import annotations

import math
import mmap
import os
import threading
import weakref
from typing import Dict, List

import numpy as np
import torch

from accdfl_amd._lib import tuning_env as _tuning_env

MODES = ("pooled", "pinned", "pageable")
_mode = os.environ.get("ACCDFL_AMD_RESULT_MEMORY", "pooled")
if _mode not in MODES:
    raise ValueError("ACCDFL_AMD_RESULT_MEMORY must be one of %s" % (MODES,))

POOL_MIN_BYTES = 1 << 20          # smaller tensors are plain torch.empty
POOL_FREE_BYTES = int(_tuning_env("ACCDFL_AMD_POOL_FREE_BYTES", str(2 << 30)))


def set_result_memory(mode: str) -> None:
    global _mode
    if mode not in MODES:
        raise ValueError("result memory mode must be one of %s" % (MODES,))
    _mode = mode


def result_memory() -> str:
    return _mode


def pin_results() -> bool:
    """Allocate a large round's result parameters page-locked (mode "pinned")."""
    return _mode == "pinned"


_NP = {torch.float32: np.float32, torch.float64: np.float64, torch.float16: np.float16,
       torch.bfloat16: np.int16, torch.int64: np.int64, torch.int32: np.int32}


class _Pool:
    """Free pre-faulted pageable blocks by size.  A tensor handed out views a numpy array over
    a block; a finalizer on that array (it lives exactly as long as the tensor's storage)
    puts the block back."""

    def __init__(self):
        self._free: Dict[int, List[mmap.mmap]] = {}
        self._free_bytes = 0
        self._lock = threading.Lock()
        # id(weakref) -> (weakref, size, block) of every block handed out: the weakref's callback returns
        # the block (a plain weakref callback, ~1 us, where weakref.finalize costs ~10 us per tensor)
        self._live: Dict[int, tuple] = {}

    def _dead(self, ref: weakref.ref):
        with self._lock:
            item = self._live.pop(id(ref), None)
        if item is not None:
            self._release(item[1], item[2])

    def _release(self, size: int, block: mmap.mmap):
        with self._lock:
            if self._free_bytes + size <= POOL_FREE_BYTES:
                self._free.setdefault(size, []).append(block)
                self._free_bytes += size
        # otherwise the block is dropped: unmapped once the dying array lets go of it

    def take(self, shape, dtype: torch.dtype, numel: "int | None" = None) -> torch.Tensor:
        if numel is None:
            numel = math.prod(shape)
        size = -(-numel * dtype.itemsize // mmap.PAGESIZE) * mmap.PAGESIZE
        with self._lock:
            blocks = self._free.get(size)
            block = blocks.pop() if blocks else None
            if block is not None:
                self._free_bytes -= size
        if block is None:
            block = mmap.mmap(-1, size)
            if hasattr(mmap, "MADV_HUGEPAGE"):
                try:
                    block.madvise(mmap.MADV_HUGEPAGE)
                except OSError:
                    pass
        arr = np.frombuffer(block, dtype=_NP[dtype], count=numel)
        ref = weakref.ref(arr, self._dead)
        with self._lock:
            self._live[id(ref)] = (ref, size, block)
        t = torch.from_numpy(arr.reshape(shape))  # the tensor keeps arr (and so the block) alive
        return t.view(torch.bfloat16) if dtype == torch.bfloat16 else t

    def free_bytes(self) -> int:
        return self._free_bytes


_pool = _Pool()


def result_tensor(shape, dtype: torch.dtype) -> torch.Tensor:
    """An uninitialised contiguous CPU tensor for a result parameter, per the mode."""
    numel = math.prod(shape)
    nbytes = numel * dtype.itemsize
    if nbytes >= POOL_MIN_BYTES:  # smaller tensors: plain torch.empty in every mode
        if _mode == "pooled" and dtype in _NP:
            return _pool.take(tuple(shape), dtype, numel)
        if _mode == "pinned" and torch.cuda.is_available():
            return torch.empty(tuple(shape), dtype=dtype, pin_memory=True)
    return torch.empty(tuple(shape), dtype=dtype)


def pool_free_bytes() -> int:
    return _pool.free_bytes()


def gpu_numa_node(device=None):
    """NUMA node of the HIP device's PCIe root (sysfs), or None when unknown."""
    if not torch.cuda.is_available():
        return None
    props = torch.cuda.get_device_properties(torch.device("cuda", 0) if device is None else device)
    try:
        bus = "%04x:%02x:%02x.0" % (getattr(props, "pci_domain_id", 0), props.pci_bus_id, props.pci_device_id)
        node = int(open("/sys/bus/pci/devices/%s/numa_node" % bus).read())
    except (AttributeError, TypeError, OSError, ValueError):
        return None
    return node if node >= 0 else None


def _cpulist(text: str):
    cpus = set()
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def bind_to_gpu_node(device=None) -> "int | None":
    """Restrict this process's CPUs to the device's NUMA node (within its current affinity), so the
    host memory it allocates afterwards — peer models, page-locked staging — is local to the GPU's
    PCIe root and the staging copies do not cross the socket link: the one-process-per-GPU
    deployment with NUMA binding (what ``numactl --cpunodebind`` does).  Returns the node, or None
    when it is unknown or would leave no CPU."""
    node = gpu_numa_node(device)
    if node is None:
        return None
    try:
        cpus = _cpulist(open("/sys/devices/system/node/node%d/cpulist" % node).read())
    except OSError:
        return None
    mine = cpus & os.sched_getaffinity(0)
    if not mine:
        return None
    try:
        os.sched_setaffinity(0, mine)
    except OSError:
        return None
    return node
