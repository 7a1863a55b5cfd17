"""PeerSlab — received peer models staged in HBM, one flat row per peer.

The reference keeps received models as CPU ``nn.Module``s in an insertion-ordered
dict (accdfl/core/model_manager.py:39-47) and only touches their bytes when the
round's aggregation runs (fedavg.py:23-25).  On MI355X the better moment to move a
model's bytes is when it ARRIVES: ``stage()`` flattens the model's parameters
(``parameters()`` order — the order fedavg.py:24 zips them in) and enqueues the H2D copy
on a dedicated copy stream, so transfers overlap the wait for the other peers.
``reduce()`` is then one device-resident launch of the libdlagg kernel over rows 0..n-1
(arrival order = summation order).

HBM layout.  fp32 / bf16 / f16 slabs are TILE-INTERLEAVED:
``buf`` is [n_tiles, capacity, tile] — row k's elements [t*tile, (t+1)*tile) sit at
``buf[t, k]``, so the tiles of every peer at one offset are adjacent and the reduce
(dla_wsum_slab_tiled) streams one region of HBM at a time instead of ``capacity`` regions
100 MB apart: 8 x 25 M fp32 130.2 us against 135.6 for separate rows, 128 x 21.3 M bf16
792 against 869 (profiles/r02d_ab_tiled.log).  ``tile`` is dla_slab_tile_elems (1-32 KiB).
A row lands in its tiles directly: each page-locked host or device source tensor is one
dla_slab_stage call on the copy stream — a 2D copy whose rows are tiles and whose destination pitch
is ``capacity`` tiles, so the copy engine writes every tile in place (round 3 staged a contiguous
device row and scattered it: 2 x the row's bytes of extra HBM traffic, one more kernel and a
row-sized buffer).  Pageable host sources go through two 16 MiB device chunks (a
contiguous H2D, then the 2D copy from the chunk: the runtime stages a 2D copy from pageable memory
one row at a time).  fp64 slabs keep one row per peer
([capacity, pitch], pitch = the parameter count rounded up to 256 bytes).  A 25 M-parameter
fp32 model is a 100 MB row; 288 GB of HBM holds ~2800 of them, so capacity is never the
constraint at accdfl's sample sizes.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
from torch import nn

from accdfl_amd import _lib
from accdfl_amd.core import wsum as _wsum

_ALIGN_BYTES = 256


class PeerSlab:

    def __init__(self, shapes: Sequence[Sequence[int]], dtype: torch.dtype, capacity: int = 8,
                 device: Optional[torch.device] = None, layout: str = "auto"):
        self.device = _wsum.require_device(device)
        self.code = _wsum.dtype_code(dtype)
        self.dtype = dtype
        self.shapes = [tuple(int(d) for d in s) for s in shapes]
        self.numels = [int(torch.Size(s).numel()) for s in self.shapes]
        self.total = sum(self.numels)
        esize = torch.empty((), dtype=dtype).element_size()
        align = _ALIGN_BYTES // esize
        self.pitch = max(align, (self.total + align - 1) // align * align)
        if layout == "auto":
            layout = "rows" if dtype == torch.float64 else "tiled"
        if layout not in ("tiled", "rows") or (layout == "tiled" and dtype == torch.float64):
            raise ValueError("PeerSlab layout must be 'tiled' (fp32/bf16/f16) or 'rows'")
        self.layout = layout
        self.capacity = max(1, int(capacity))
        self.tile = 0
        self.buf = self._alloc(self.capacity)
        self.n = 0
        self.copy_stream = torch.cuda.Stream(self.device)
        self._bounce = [None, None]
        self._bounce_ev = [None, None]
        self._dev_chunks = None    # device staging of pageable host sources (_put_pageable)
        self._held: List[torch.Tensor] = []  # page-locked sources of the stage call in progress
        # page-locked host sources of copies still in flight, with the copy stream's event after them:
        # dla_slab_stage's DMAs are not seen by torch's pinned-memory allocator (a torch copy_ records an
        # event there), so the slab keeps the tensors — and their blocks out of the allocator's reuse —
        # until the copy stream has passed them
        self._inflight: List[tuple] = []
        self._h_out = None
        self._flat = None          # device result of reduce_into (reused every round)
        self._plan = None          # prepared launch over (rows 0..n-1, _flat)
        self._plan_key = None

    def _alloc(self, capacity: int) -> torch.Tensor:
        if self.layout == "rows":
            return torch.empty((capacity, self.pitch), dtype=self.dtype, device=self.device)
        self.tile = max(1, _lib.slab_tile_elems(self.code, capacity, self.total))
        n_tiles = max(1, -(-self.total // self.tile))
        return torch.empty((n_tiles, capacity, self.tile), dtype=self.dtype, device=self.device)

    def _tiles_of(self, buf: torch.Tensor, k: int) -> torch.Tensor:
        """Row k of a tiled slab as a [n_tiles, tile] view."""
        return buf[:, k, :]

    def row(self, k: int) -> torch.Tensor:
        """Row k's ``total`` elements as a contiguous device tensor (a copy for tiled slabs)."""
        if self.layout == "rows":
            return self.buf[k, : self.total]
        return self._tiles_of(self.buf, k).reshape(-1)[: self.total]

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
        cur = torch.cuda.current_stream(self.device)
        self.copy_stream.wait_stream(cur)
        with torch.cuda.stream(self.copy_stream):
            old, old_tile = self.buf, self.tile
            new = self._alloc(cap)  # a tiled slab may change its tile with the row count
            if self.n:
                if self.layout == "rows":
                    new[: self.n].copy_(old[: self.n])
                elif self.tile == old_tile:
                    new[:, : self.n, :].copy_(old[:, : self.n, :])
                else:
                    for k in range(self.n):
                        flat = self._tiles_of(old, k).reshape(-1)[: self.total].contiguous()
                        _lib.slab_stage(self.code, new.data_ptr(), self.tile, cap, new.shape[0], k, 0, flat.data_ptr(),
                                        self.total, int(self.copy_stream.cuda_stream))
                        flat.record_stream(self.copy_stream)
        old.record_stream(self.copy_stream)
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

    # Pageable host sources of a tiled slab go through device chunks of this size (two, reused in
    # stream order): a contiguous H2D, then a 2D D2D copy into the tiles.  A 2D copy straight from
    # pageable memory is staged by the runtime row by row — one tile at a time — and moved a 100 MB
    # wire payload at 5.7 GB/s (bench.py wire_ingress, profiles/r04a-r04g) against 51.8 for round 3's
    # contiguous H2D; the D2D pass costs ~2 % (2.1 TB/s, profiles/r04a/copy_probe.log).
    PAGEABLE_CHUNK_BYTES = 16 << 20

    def _put(self, row: int, off: int, src: torch.Tensor, n: int):
        """``n`` elements at ``src`` (host or this device) -> row ``row`` from element ``off`` on, on the
        copy stream.  Tiled slabs: dla_slab_stage, one 2D copy that writes every tile in place (from
        page-locked host or device memory; pageable host memory through _put_pageable)."""
        if self.layout == "rows":
            self.buf[row, off:off + n].copy_(src.view(-1)[:n], non_blocking=src.device.type == "cpu" and src.is_pinned())
            return
        if src.device.type == "cpu":
            if not src.is_pinned():
                self._put_pageable(row, off, src, n)
                return
            self._held.append(src)
        _lib.slab_stage(self.code, self.buf.data_ptr(), self.tile, self.capacity, self.buf.shape[0], row, off,
                        src.data_ptr(), n, int(self.copy_stream.cuda_stream))

    def _put_pageable(self, row: int, off: int, src: torch.Tensor, n: int):
        chunk = max(1, self.PAGEABLE_CHUNK_BYTES // self.buf.element_size())
        if self._dev_chunks is None:
            self._dev_chunks = [torch.empty(chunk, dtype=self.dtype, device=self.device) for _ in range(2)]
        flat = src.view(-1)
        with torch.cuda.stream(self.copy_stream):
            for i, s0 in enumerate(range(0, n, chunk)):
                m = min(chunk, n - s0)
                buf = self._dev_chunks[i & 1][:m]
                buf.copy_(flat[s0:s0 + m], non_blocking=True)  # pageable: consumed before this returns
                _lib.slab_stage(self.code, self.buf.data_ptr(), self.tile, self.capacity, self.buf.shape[0], row,
                                off + s0, buf.data_ptr(), m, int(self.copy_stream.cuda_stream))

    def _release_inflight(self):
        """Drop the page-locked sources whose copies the copy stream has passed."""
        while self._inflight and self._inflight[0][0].query():
            self._inflight.pop(0)

    def _stage_flat_list(self, flat: List[torch.Tensor]) -> int:
        self._release_inflight()
        self._held: List[torch.Tensor] = []
        try:
            return self._stage_flat_list_held(flat)
        finally:
            if self._held:
                ev = torch.cuda.Event()
                ev.record(self.copy_stream)
                self._inflight.append((ev, self._held))
            self._held = []

    def _stage_flat_list_held(self, flat: List[torch.Tensor]) -> int:
        row = self.n
        if row >= self.capacity:
            self._grow(row + 1)
        cur = torch.cuda.current_stream(self.device)
        self.copy_stream.wait_stream(cur)
        esize = self.buf.element_size()
        if all(t.device.type == "cpu" for t in flat):
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
                        self._put(row, run_start, bounce[run_start:off], off - run_start)
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
                        # straight from where the tensor lives: pageable (no host copy) or a page-locked
                        # ingress buffer (async; the caller keeps it until copy_stream passes)
                        self._put(row, off, t, t.numel())
                    off += t.numel()
                if bounce is not None:
                    ev = torch.cuda.Event()
                    ev.record(self.copy_stream)
                    self._bounce_ev[slot] = ev
        else:
            with torch.cuda.stream(self.copy_stream):
                off = 0
                for t in flat:
                    src = t if t.device == self.device else t.to(self.device, non_blocking=True)
                    src = src.contiguous()
                    self._put(row, off, src, src.numel())
                    if src is not t:
                        src.record_stream(self.copy_stream)  # a temporary: freed only after its copy
                    off += t.numel()
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
        if self.layout == "rows":
            return _wsum.wsum_rows(self.buf, weights, self.total, out=out)
        if out is None:
            out = torch.empty(self.total, dtype=self.dtype, device=self.device)
        if out.device != self.device or out.dtype != self.dtype or out.numel() < self.total or not out.is_contiguous():
            raise ValueError("out must be a contiguous %s tensor of >= %d elements on %s"
                             % (self.dtype, self.total, self.device))
        _lib.wsum_slab_tiled_ptr(self.code, self.buf.data_ptr(), self.tile, self.capacity, weights, self.total,
                                 out.data_ptr(), int(cur.cuda_stream))
        return out

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
        if self.layout == "tiled":
            return self.reduce(weights, out=self._flat)[: self.total]
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
        large = self.total * self.buf.element_size() >= 8 << 20
        if all(p.is_contiguous() and p.device.type == "cpu" for p in params) and (
                all(p.is_pinned() for p in params) or large):
            # D2H straight into the result: page-locked tensors (result-memory mode "pinned") or,
            # for large models, pageable ones through the runtime's staging (core/host_memory.py)
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
