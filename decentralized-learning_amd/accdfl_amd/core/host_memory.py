"""Host memory of the averaged model's CPU parameters.

The reference returns ``deepcopy(models[0])`` with ordinary (pageable) CPU tensors
(accdfl/core/gradient_aggregation/fedavg.py:20), and callers keep that model: the simulator
holds one per node.  The reduce's D2H has to land in those tensors.  Three ways, chosen by
``ACCDFL_AMD_RESULT_MEMORY`` or ``set_result_memory``:

* ``registered`` (default): the result's tensors are ordinary pageable memory, exactly like
  the reference's.  For the duration of one aggregation the large ones (>= 1 MiB) are
  page-locked in place with ``hipHostRegister`` so the D2H writes them directly (DMA), then
  unlocked — nothing stays page-locked after the call, however many results are kept.
* ``pinned``: the result's tensors are allocated page-locked (``is_pinned()``).  They stay
  page-locked for the model's lifetime and torch's caching host allocator keeps freed blocks
  page-locked too, so host page-locked memory grows with the number of results kept.
* ``pageable``: plain pageable tensors, D2H through the runtime's own staging.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Iterable, List

import torch

MODES = ("registered", "pinned", "pageable")
_mode = os.environ.get("ACCDFL_AMD_RESULT_MEMORY", "registered")
if _mode not in MODES:
    raise ValueError("ACCDFL_AMD_RESULT_MEMORY must be one of %s" % (MODES,))

REGISTER_MIN_BYTES = 1 << 20
_hip = None


def set_result_memory(mode: str) -> None:
    global _mode
    if mode not in MODES:
        raise ValueError("result memory mode must be one of %s" % (MODES,))
    _mode = mode


def result_memory() -> str:
    return _mode


def pin_results() -> bool:
    """Allocate the result's CPU parameters page-locked (mode "pinned")."""
    return _mode == "pinned"


def _runtime():
    """The HIP runtime torch already loaded (same soname: one runtime per process)."""
    global _hip
    if _hip is None:
        torch.cuda.init()
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
        _hip.hipHostRegister.restype = ctypes.c_int
        _hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
        _hip.hipHostUnregister.restype = ctypes.c_int
        _hip.hipGetLastError.restype = ctypes.c_int
    return _hip


@contextlib.contextmanager
def registered(tensors: Iterable[torch.Tensor]):
    """Page-lock the large, contiguous, pageable CPU tensors among ``tensors`` for the
    duration of the block (mode "registered"; otherwise a no-op).  A tensor the runtime
    refuses to register simply stays pageable (its copy goes through the runtime's staging)."""
    done: List[int] = []
    if _mode == "registered":
        hip = _runtime()
        seen = set()
        for t in tensors:
            if (t.device.type != "cpu" or not t.is_contiguous() or t.is_pinned()
                    or t.numel() * t.element_size() < REGISTER_MIN_BYTES):
                continue
            ptr = t.data_ptr()
            if ptr in seen:
                continue
            seen.add(ptr)
            if hip.hipHostRegister(ptr, t.numel() * t.element_size(), 0) == 0:
                done.append(ptr)
            else:
                hip.hipGetLastError()  # clear the runtime's sticky last error: the copy just stays staged
    try:
        yield done
    finally:
        if done:
            hip = _runtime()
            for ptr in done:
                hip.hipHostUnregister(ptr)
