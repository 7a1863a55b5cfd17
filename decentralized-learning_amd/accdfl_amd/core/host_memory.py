"""Host memory of the averaged model's CPU parameters.

The reference returns ``deepcopy(models[0])`` with ordinary (pageable) CPU tensors
(accdfl/core/gradient_aggregation/fedavg.py:20), and callers keep that model: the simulator
holds one per node.  The reduce's D2H has to land in those tensors.  Two modes, chosen by
``ACCDFL_AMD_RESULT_MEMORY`` or ``set_result_memory``:

* ``pageable`` (default): the result's tensors are ordinary pageable memory, exactly like the
  reference's; the D2H goes through the HIP runtime's own staging.  Nothing stays page-locked
  however many results a caller keeps.
* ``pinned``: the result's tensors of a large round are allocated page-locked
  (``is_pinned()``) and the D2H writes them directly.  Faster (8 x 25 M fp32 host-inclusive
  round 16.6-17.4 ms against 21.8-22.4), but they stay page-locked for the model's lifetime,
  and torch's caching host allocator keeps freed blocks page-locked too, so page-locked host
  memory grows with the number of results kept.

Locking the pageable result in place for the duration of the D2H (``hipHostRegister``) was
measured too and bought nothing over ``pageable`` (21.8-22.1 ms): the cost of a fresh
pageable result is faulting its pages in, which the reference's deepcopy pays as well
(profiles/r02d_result_memory.log).
"""
from __future__ import annotations

import os

MODES = ("pageable", "pinned")
_mode = os.environ.get("ACCDFL_AMD_RESULT_MEMORY", "pageable")
if _mode not in MODES:
    raise ValueError("ACCDFL_AMD_RESULT_MEMORY must be one of %s" % (MODES,))


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
