"""Teacher-logit aggregation for knowledge distillation (§8 f4).

Reference: scripts/distill.py:124-129 averages the N teachers' logits sample by sample::

    for sample_ind in range(len(logits[0])):
        predictions = [logits[n][sample_ind] for n in range(args.peers)]
        aggregated_predictions.append(torch.mean(torch.stack(predictions), dim=0))

— one stack + one reduction launch per sample.  Here the whole batch is one
``dla_mean`` launch over N teacher buffers of S x C logits: a sequential sum in
list order from +0, then a correctly rounded division by N (include/dlagg.h).
torch's own sum order is implementation-defined (and the reference ran it on CUDA),
so parity with ``torch.mean`` is within ``N * 2^-23 * sum|p| / N`` per element (f32);
against the sequential-sum oracle it is bit-exact (tests/test_gpu_parity.py).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from accdfl_amd import _lib
from accdfl_amd.core import wsum as _wsum


def mean_logits(teacher_logits: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Element-wise mean over N same-shaped device tensors (e.g. N teachers' [S, C]
    logits): ``torch.mean(torch.stack(teacher_logits), dim=0)`` as one HIP launch."""
    n = len(teacher_logits)
    if n < 1:
        raise RuntimeError("mean of an empty list")  # torch.stack([]) raises too
    t0 = teacher_logits[0]
    device = _wsum.require_device(t0.device)
    if t0.dtype not in (torch.float32, torch.float64):
        raise TypeError("mean_logits: float32 or float64 logits, got %s" % t0.dtype)
    for k, t in enumerate(teacher_logits):
        if t.shape != t0.shape or t.dtype != t0.dtype or t.device != device or not t.is_contiguous():
            raise ValueError("teacher %d: logits must share shape/dtype/device and be contiguous" % k)
    if out is None:
        out = torch.empty_like(t0)
    _lib.mean_ptrs(_wsum.dtype_code(t0.dtype), [t.data_ptr() for t in teacher_logits], t0.numel(), out.data_ptr(),
                   int(torch.cuda.current_stream(device).cuda_stream))
    return out


def aggregate_predictions(logits: Sequence[Sequence[torch.Tensor]]) -> List[torch.Tensor]:
    """Drop-in for distill.py:124-129: ``logits[n]`` is teacher n's list of per-sample
    [C] outputs; returns the per-sample means (views of one [S, C] result)."""
    device = _wsum.require_device(logits[0][0].device if logits and logits[0] else None)
    stacked = [torch.stack([x.to(device) for x in per_teacher]).contiguous() for per_teacher in logits]
    return list(mean_logits(stacked).unbind(0))
