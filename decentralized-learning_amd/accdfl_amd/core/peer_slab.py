"""PeerSlab — received peer models staged in HBM, one flat row per peer.

The reference keeps received models as CPU ``nn.Module``s in an insertion-ordered
dict (accdfl/core/model_manager.py:39-47) and only touches their bytes when the
round's aggregation runs (fedavg.py:23-25).  On MI355X the better moment to move a
model's bytes is when it ARRIVES: ``stage()`` flattens the model's parameters
(``parameters()`` order — the order fedavg.py:24 zips them in) into a pinned bounce
buffer and enqueues the H2D copy on a dedicated copy stream, so transfers overlap
the wait for the other peers.  ``reduce()`` is then one device-resident launch of
the libdlagg kernel over rows 0..n-1 (arrival order = summation order).

HBM layout: ``buf`` is a row-major [capacity, pitch] slab of the parameter dtype;
``pitch`` is the flat parameter count rounded up to 256 bytes so every row starts
16-byte aligned (the kernel's dwordx4 path).  A 25 M-parameter fp32 model is a
100 MB row; 288 GB of HBM holds ~2800 of them, so capacity is never the constraint
at accdfl's sample sizes.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
from torch import nn

from accdfl_amd import _lib
from accdfl_amd.core import host_memory as _host_memory
from accdfl_amd.core import wsum as _wsum

_ALIGN_BYTES = 256


class PeerSlab:

    def __init__(self, shapes: Sequence[Sequence[int]], dtype: torch.dtype, capacity: int = 8,
                 device: Optional[torch.device] = None):
        self.device = _wsum.require_device(device)
        _wsum.dtype_code(dtype)
        self.dtype = dtype
        self.shapes = [tuple(int(d) for d in s) for s in shapes]
        self.numels = [int(torch.Size(s).numel()) for s in self.shapes]
        self.total = sum(self.numels)
        esize = torch.empty((), dtype=dtype).element_size()
        align = _ALIGN_BYTES // esize
        self.pitch = max(align, (self.total + align - 1) // align * align)
        self.capacity = max(1, int(capacity))
        self.buf = torch.empty((self.capacity, self.pitch), dtype=dtype, device=self.device)
        self.n = 0
        self.copy_stream = torch.cuda.Stream(self.device)
        self._bounce = [None, None]
        self._bounce_ev = [None, None]
        self._h_out = None
        self._flat = None          # device result of reduce_into (reused every round)
        self._plan = None          # prepared launch over (rows 0..n-1, _flat)
        self._plan_key = None

    # ------------------------------------------------------------------ creation
    @classmethod
    def for_model(cls, model: nn.Module, capacity: int = 8, device: Optional[torch.device] = None) -> "PeerSlab":
        params = list(model.parameters())
        dtypes = {p.dtype for p in params}
        if len(dtypes) != 1:
            raise TypeError("PeerSlab holds one parameter dtype; model has %s" % sorted(map(str, dtypes)))
        return cls([p.shape for p in params], params[0].dtype, capacity, device)

    def matches(self, params: Sequence[torch.Tensor]) -> bool:
        return (len(params) == len(self.shapes)
                and all(tuple(p.shape) == s and p.dtype == self.dtype for p, s in zip(params, self.shapes)))

    def uniform_with(self, models: Sequence[nn.Module]) -> bool:
        """True when rows 0..n-1 hold exactly ``models`` (same count, same layout)."""
        return len(models) == self.n and all(self.matches(list(m.parameters())) for m in models)

    # ------------------------------------------------------------------- staging
    def _grow(self, rows: int):
        cap = max(rows, 2 * self.capacity)
        new = torch.empty((cap, self.pitch), dtype=self.dtype, device=self.device)
        cur = torch.cuda.current_stream(self.device)
        self.copy_stream.wait_stream(cur)
        with torch.cuda.stream(self.copy_stream):
            if self.n:
                new[: self.n].copy_(self.buf[: self.n])
        self.buf.record_stream(self.copy_stream)
        self.buf = new
        self.capacity = cap

    def _bounce_buffer(self, slot: int) -> torch.Tensor:
        ev = self._bounce_ev[slot]
        if ev is not None:
            ev.synchronize()  # the H2D that last read this pinned buffer has finished
        if self._bounce[slot] is None:
            self._bounce[slot] = torch.empty(self.pitch, dtype=self.dtype, pin_memory=True)
        return self._bounce[slot]

    def stage(self, model_or_params) -> int:
        """Append one peer model (nn.Module or parameter list) as the next row; returns it."""
        params = list(model_or_params.parameters()) if isinstance(model_or_params, nn.Module) else list(
            model_or_params)
        if not self.matches(params):
            raise ValueError("PeerSlab.stage: parameter layout differs from the slab's")
        flat = [p.detach().reshape(-1) for p in params]
        return self._stage_flat_list(flat)

    def stage_flat(self, flat: torch.Tensor) -> int:
        """Append a peer given as one flat tensor of ``total`` elements."""
        if flat.numel() != self.total or flat.dtype != self.dtype:
            raise ValueError("PeerSlab.stage_flat: need %d elements of %s" % (self.total, self.dtype))
        return self._stage_flat_list([flat.detach().reshape(-1)])

    # Tensors at least this large go H2D straight from where they live (e.g. the wire
    # payload): ROCm's pageable H2D runs at the pinned rate on MI355X hosts (14.2 vs 13.9 ms
    # per 800 MB), so the bounce copy would only add a host memcpy.  Runs of smaller
    # tensors are packed into the pinned bounce buffer and sent as one copy.
    DIRECT_BYTES = 1 << 20

    def _stage_flat_list(self, flat: List[torch.Tensor]) -> int:
        row = self.n
        if row >= self.capacity:
            self._grow(row + 1)
        cur = torch.cuda.current_stream(self.device)
        self.copy_stream.wait_stream(cur)
        if all(t.device.type == "cpu" for t in flat):
            esize = self.buf.element_size()
            slot = row & 1
            bounce = None
            run_start = None  # element offset where the current run of small tensors begins
            off = 0
            pending = ([], [], [])  # (dst, src, bytes) of the run: one native batched memcpy
            with torch.cuda.stream(self.copy_stream):
                for t in flat + [None]:
                    small = t is not None and t.numel() * esize < self.DIRECT_BYTES
                    if not small and run_start is not None:  # flush the run of small tensors
                        _lib.host_copy_batch(*pending)
                        pending = ([], [], [])
                        self.buf[row, run_start:off].copy_(bounce[run_start:off], non_blocking=True)
                        run_start = None
                    if t is None:
                        break
                    if small:
                        if bounce is None:
                            bounce = self._bounce_buffer(slot)
                        if run_start is None:
                            run_start = off
                        pending[0].append(bounce.data_ptr() + off * esize)
                        pending[1].append(t.data_ptr())
                        pending[2].append(t.numel() * esize)
                    else:
                        self.buf[row, off:off + t.numel()].copy_(t)  # pageable H2D, no host copy
                    off += t.numel()
                if bounce is not None:
                    ev = torch.cuda.Event()
                    ev.record(self.copy_stream)
                    self._bounce_ev[slot] = ev
        else:
            dst = self.buf[row, : self.total]
            with torch.cuda.stream(self.copy_stream):
                src = [t.to(self.device, non_blocking=True) for t in flat]
                if len(src) == 1:
                    dst.copy_(src[0])
                else:
                    torch.cat(src, out=dst)
        self.n = row + 1
        return row

    def reset(self):
        """Start a new round (rows are overwritten by the next stage() calls)."""
        self.n = 0

    # -------------------------------------------------------------------- reduce
    def reduce(self, weights: Optional[Sequence[float]] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """FedAvg over the staged rows in arrival order (fedavg.py:14-25)."""
        n = self.n
        if not weights:
            weights = [float(1. / n) for _ in range(n)]
        else:
            assert len(weights) == n
        if n < 1:
            raise IndexError("list index out of range")
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(self.copy_stream)
        return _wsum.wsum_rows(self.buf, weights, self.total, out=out)

    def _offsets(self) -> List[int]:
        offs, o = [], 0
        for m in self.numels:
            offs.append(o)
            o += m
        return offs

    def unflatten(self, flat: torch.Tensor) -> List[torch.Tensor]:
        return [t.view(s) for t, s in zip(torch.split(flat[: self.total], self.numels), self.shapes)]

    def _reduce_planned(self, weights: Optional[Sequence[float]]) -> torch.Tensor:
        """reduce() into the slab's own result buffer through a cached dla_plan (the
        same rows and output every round: only the launch is paid)."""
        n = self.n
        if not weights:
            weights = [float(1. / n) for _ in range(n)]
        else:
            assert len(weights) == n
        if n < 1:
            raise IndexError("list index out of range")
        if self._flat is None:
            self._flat = torch.empty(self.pitch, dtype=self.dtype, device=self.device)
        key = (n, self.buf.data_ptr(), self._flat.data_ptr())
        if self._plan_key != key:
            ptrs = [self.buf[k].data_ptr() for k in range(n)]
            self._plan = _lib.Plan(_wsum.dtype_code(self.dtype), ptrs, weights, self.total, self._flat.data_ptr())
            self._plan_key = key
        else:
            self._plan.set_weights(weights)
        cur = torch.cuda.current_stream(self.device)
        cur.wait_stream(self.copy_stream)
        self._plan.launch(int(cur.cuda_stream))
        return self._flat[: self.total]

    def reduce_into(self, params: Sequence[torch.Tensor], weights: Optional[Sequence[float]] = None) -> None:
        """Reduce and write the result into ``params`` (CPU or device tensors)."""
        flat = self._reduce_planned(weights)
        if all(p.device == self.device for p in params):
            for p, v in zip(params, self.unflatten(flat)):
                p.copy_(v)
            return
        large = self.total * self.buf.element_size() >= 8 * _host_memory.REGISTER_MIN_BYTES
        if all(p.is_contiguous() and p.device.type == "cpu" for p in params) and (
                all(p.is_pinned() for p in params) or (large and _host_memory.result_memory() != "pinned")):
            # D2H straight into the result: page-locked tensors, or (large models) tensors
            # page-locked for this call only (core/host_memory.py) / staged by the runtime
            with _host_memory.registered(params):
                for p, v in zip(params, torch.split(flat, self.numels)):
                    p.view(-1).copy_(v, non_blocking=True)
                torch.cuda.current_stream(self.device).synchronize()
            return
        if all(p.is_contiguous() and p.device.type == "cpu" for p in params):  # small rounds: one D2H,
            if self._h_out is None or self._h_out.numel() < self.total:      # one native host scatter
                self._h_out = torch.empty(self.pitch, dtype=self.dtype, pin_memory=True)
            h = self._h_out[: self.total]
            h.copy_(flat, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            esize = h.element_size()
            srcs = [h.data_ptr() + o * esize for o in self._offsets()]
            _lib.host_copy_batch([p.data_ptr() for p in params], srcs, [m * esize for m in self.numels])
            return
        if self._h_out is None or self._h_out.numel() < self.total:
            self._h_out = torch.empty(self.pitch, dtype=self.dtype, pin_memory=True)
        h = self._h_out[: self.total]
        h.copy_(flat, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        for p, v in zip(params, [t.view(s) for t, s in zip(torch.split(h, self.numels), self.shapes)]):
            p.copy_(v)
