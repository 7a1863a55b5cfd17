"""Torch-facing wrappers of the libdlagg reduce (device tensors in, device tensors out).

The arithmetic is the reference's FedAvg inner loop
(accdfl/core/gradient_aggregation/fedavg.py:21-25) executed by the gfx950 kernel in
csrc/dlagg.hip; these helpers only validate tensors, pick the stream and pass raw
pointers across the C ABI.  Work is enqueued on the current HIP stream of the
tensors' device and is NOT synchronised (torch stream semantics).
"""
from __future__ import annotations

import os
import threading
from typing import List, Optional, Sequence

import torch

from .. import _lib

_CODES = {
    torch.float32: _lib.DLA_F32,
    torch.bfloat16: _lib.DLA_BF16,
    torch.float16: _lib.DLA_F16,
    torch.float64: _lib.DLA_F64,
}

SUPPORTED_DTYPES = tuple(_CODES)
_ESIZE = {torch.float32: 4, torch.bfloat16: 2, torch.float16: 2, torch.float64: 8}


def dtype_code(dtype: torch.dtype) -> int:
    try:
        return _CODES[dtype]
    except KeyError:
        raise TypeError("accdfl_amd FedAvg supports float32/bfloat16/float16/float64 parameters, got %s" % dtype)


def require_device(device: Optional[torch.device] = None) -> torch.device:
    """The HIP device the reduce runs on; raises when there is none (no CPU fallback)."""
    if not torch.cuda.is_available():
        raise RuntimeError("accdfl_amd: no HIP device visible — the aggregation reduce runs only on the GPU "
                           "(MI355X); there is no CPU fallback")
    if device is None or device.type != "cuda":
        return torch.device("cuda", torch.cuda.current_device())
    return device


def _stream_ptr(device: torch.device, stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return int(s.cuda_stream)


def _check_dev(t: torch.Tensor, device: torch.device, what: str):
    if t.device != device:
        raise ValueError("%s is on %s, expected %s" % (what, t.device, device))
    if not t.is_contiguous():
        raise ValueError("%s must be contiguous" % what)


def wsum(peers: Sequence[torch.Tensor], weights: Sequence[float], out: Optional[torch.Tensor] = None,
         stream: Optional[torch.cuda.Stream] = None, cfg: Optional[_lib.LaunchCfg] = None) -> torch.Tensor:
    """out = FedAvg(peers, weights) element-wise, one device buffer per peer.

    ``peers``: N contiguous device tensors of one dtype and numel (list order =
    summation order); ``weights``: N numbers (already defaulted).  ``out`` may alias
    ``peers[0]``.
    """
    n = len(peers)
    if n < 1:
        raise IndexError("list index out of range")
    if len(weights) != n:
        raise AssertionError("len(weights) != len(peers)")
    p0 = peers[0]
    device = require_device(p0.device)
    code = dtype_code(p0.dtype)
    numel = p0.numel()
    for k, p in enumerate(peers):
        _check_dev(p, device, "peer %d" % k)
        if p.dtype != p0.dtype or p.numel() != numel:
            raise ValueError("peer %d: dtype/numel %s/%d differs from peer 0 %s/%d" % (k, p.dtype, p.numel(),
                                                                                        p0.dtype, numel))
    if out is None:
        out = torch.empty_like(p0)
    _check_dev(out, device, "out")
    if out.dtype != p0.dtype or out.numel() != numel:
        raise ValueError("out dtype/numel mismatch")
    _lib.wsum_ptrs(code, [p.data_ptr() for p in peers], weights, numel, out.data_ptr(),
                   _stream_ptr(device, stream), cfg)
    return out


def wsum_mixed(peers: Sequence[torch.Tensor], weights: Sequence[float], out: torch.Tensor,
               stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """out = FedAvg(peers, weights) when the peers do not share one dtype (dla_wsum_mixed): each
    product is rounded in its peer's dtype and each sum in ``out``'s (peers[0]'s) dtype after
    promotion, as ``c1.add_(w * p1)`` (fedavg.py:25) does for a peer of another dtype."""
    n = len(peers)
    if n < 1:
        raise IndexError("list index out of range")
    if len(weights) != n:
        raise AssertionError("len(weights) != len(peers)")
    device = require_device(out.device)
    _check_dev(out, device, "out")
    numel = out.numel()
    for k, p in enumerate(peers):
        _check_dev(p, device, "peer %d" % k)
        if p.numel() != numel:
            raise ValueError("peer %d: numel %d differs from out's %d" % (k, p.numel(), numel))
    if peers[0].dtype != out.dtype:
        raise ValueError("peer 0 (models[0]) must have out's dtype")
    _lib.wsum_mixed_ptrs(dtype_code(out.dtype), [dtype_code(p.dtype) for p in peers], [p.data_ptr() for p in peers],
                         weights, numel, out.data_ptr(), _stream_ptr(device, stream))
    return out


def wsum_rows(slab: torch.Tensor, weights: Sequence[float], n_elems: Optional[int] = None,
              out: Optional[torch.Tensor] = None, stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """FedAvg over the first len(weights) rows of a 2-D device slab [rows, pitch]."""
    if slab.dim() != 2 or slab.stride(1) != 1:
        raise ValueError("slab must be a 2-D row-major tensor")
    n = len(weights)
    if n < 1 or n > slab.shape[0]:
        raise ValueError("need 1 <= len(weights) <= slab rows")
    device = require_device(slab.device)
    if slab.device != device:
        raise ValueError("slab is not on a HIP device")
    code = dtype_code(slab.dtype)
    n_elems = slab.shape[1] if n_elems is None else int(n_elems)
    if out is None:
        out = torch.empty(n_elems, dtype=slab.dtype, device=device)
    _check_dev(out, device, "out")
    if out.numel() < n_elems or out.dtype != slab.dtype:
        raise ValueError("out too small or wrong dtype")
    _lib.wsum_slab_ptr(code, slab.data_ptr(), slab.stride(0), weights, n, n_elems, out.data_ptr(),
                       _stream_ptr(device, stream))
    return out


def wsum_multi(peer_params: Sequence[Sequence[torch.Tensor]], weights: Sequence[float],
               outs: Sequence[torch.Tensor], stream: Optional[torch.cuda.Stream] = None) -> None:
    """Multi-tensor FedAvg: outs[i] = FedAvg([peer_params[k][i] for k], weights).

    All tensors device-resident and contiguous; outs[i] may alias peer_params[0][i].
    One dtype per call (the caller groups tensors by dtype).
    """
    if not outs:
        return
    n = len(peer_params)
    device = require_device(outs[0].device)
    ptrs: List[int] = []
    for i, o in enumerate(outs):
        _check_dev(o, device, "out %d" % i)
        if o.dtype != outs[0].dtype:
            raise ValueError("wsum_multi: one dtype per call")
        for k in range(n):
            p = peer_params[k][i]
            _check_dev(p, device, "peer %d tensor %d" % (k, i))
            if p.numel() != o.numel() or p.dtype != o.dtype:
                raise ValueError("peer %d tensor %d: numel/dtype mismatch" % (k, i))
            ptrs.append(p.data_ptr())
    wsum_multi_ptrs(outs[0].dtype, ptrs, [o.data_ptr() for o in outs], [o.numel() for o in outs], weights, device,
                    stream)


# Rounds of at least MULTI_TABLE_MIN_PEERS peers — or of more than 8 peers moving at least
# MULTI_TABLE_MIN_BYTES — reduce every aligned tensor in one launch per 128-peer pass through a
# device-side pointer table (dla_wsum_multi_table); other rounds pack up to 32 small tensors per
# launch with the pointers in the kernel arguments (dla_wsum_multi), which needs no table copy.
# Interleaved A/B on MI355X (profiles/r03e/, us, table / kernel-argument path, flat slab beside):
# 128 x ResNet-34 bf16 865 / 1851 (813); 64 x ResNet-8 f32 219 / 310 (192); 64 x GNLeNet 14 / 48
# (4.3); 16 x ResNet-34 bf16 (724 MB) 134 / 165 (106); but 32 x FEMNIST (223 MB) 41.3 / 35.2 (32.1)
# and 8 x GNLeNet 13.0 / 6.3 (3.3), where the table's copy costs more than it saves.
MULTI_TABLE_MIN_PEERS = int(_lib.tuning_env("ACCDFL_AMD_MULTI_TABLE_MIN_PEERS", "33"))
MULTI_TABLE_MIN_BYTES = 256 << 20


class _TableRing:
    """Page-locked host + device buffers for dla_wsum_multi_table's table, SLOTS slots per device used
    round-robin.  A slot is refilled only after the stream that last read it has passed that call, so
    back-to-back rounds never overwrite a table still being copied or read.  The guard is one event per
    FENCE_EVERY calls (recorded after the last of them, on their stream), not one per call: an event
    recorded between two kernels of a stream costs ~3 us of GPU time (profiles/r05e: 124.8 -> 127.7 us
    per back-to-back headline reduce); a slot is reused SLOTS calls after its last use, by when the
    event after it has been recorded (or is recorded then)."""

    SLOTS = 8
    FENCE_EVERY = 4

    def __init__(self, device: torch.device):
        self.device = device
        self.slots = [None] * self.SLOTS  # (host uint8, device uint8)
        self.fence = [None] * self.SLOTS  # event recorded after the slot's last use, or None
        self.busy = [False] * self.SLOTS  # taken and not yet done (another thread's call in flight)
        self.pending = []                 # (slot, stream) used since the last fence
        self.i = 0
        self.lock = threading.Lock()

    def _fence_locked(self):
        """Record the event covering every pending slot (one per stream they ran on)."""
        evs = {}
        for idx, st in self.pending:
            ev = evs.get(st.cuda_stream)
            if ev is None:
                ev = evs[st.cuda_stream] = torch.cuda.Event()
                ev.record(st)
            self.fence[idx] = ev
        self.pending = []

    def take(self, nbytes: int):
        """(slot index, host buffer, device buffer); the caller passes the index to done()."""
        with self.lock:
            for _ in range(self.SLOTS):
                self.i = (self.i + 1) % self.SLOTS
                if not self.busy[self.i]:
                    break
            else:
                raise RuntimeError("wsum_multi_table: more than %d concurrent calls on %s" % (self.SLOTS, self.device))
            idx = self.i
            self.busy[idx] = True
            if any(k == idx for k, _ in self.pending):
                self._fence_locked()
            ev, slot = self.fence[idx], self.slots[idx]
        if ev is not None:
            ev.synchronize()
        if slot is None or slot[0].numel() < nbytes:
            size = max(nbytes, 64 << 10)
            size = 1 << (size - 1).bit_length()
            slot = (torch.empty(size, dtype=torch.uint8, pin_memory=True),
                    torch.empty(size, dtype=torch.uint8, device=self.device))
            self.slots[idx] = slot
        return idx, slot[0], slot[1]

    def done(self, idx: int, stream: torch.cuda.Stream):
        with self.lock:
            self.busy[idx] = False
            if self.pending and self.pending[-1][1].cuda_stream != stream.cuda_stream:
                self._fence_locked()
            self.pending.append((idx, stream))
            if len(self.pending) >= self.FENCE_EVERY:
                self._fence_locked()


_rings = {}
_rings_lock = threading.Lock()


_table_bytes = {}  # (n_tensors, n_peers) -> dla_wsum_multi_table_bytes


def wsum_multi_ptrs(dtype: torch.dtype, ptrs, out_ptrs, numels, weights: Sequence[float], device: torch.device,
                    stream: Optional[torch.cuda.Stream] = None, acc_in: bool = False,
                    total_elems: Optional[int] = None) -> None:
    """wsum_multi on raw pointers the caller has validated (device-resident, contiguous, one dtype,
    numels[i] elements each; ptrs tensor-major [n_tensors * n_peers]).  Rounds of more than
    MULTI_TABLE_MIN_PEERS - 1 peers go through dla_wsum_multi_table (one launch per 128-peer pass).
    ``total_elems``: sum(numels) when the caller knows it (a device round's flat plan: no pass over a
    ctypes array of numels on the launch path)."""
    code = dtype_code(dtype)
    n = len(weights)
    s = stream if stream is not None else torch.cuda.current_stream(device)
    table = acc_in or n >= MULTI_TABLE_MIN_PEERS or (
        n > 8 and (n + 1) * (sum(numels) if total_elems is None else total_elems) * _ESIZE[dtype]
        >= MULTI_TABLE_MIN_BYTES)
    if table and (dtype != torch.float64 or acc_in):  # fp64 folds per tensor inside the table call
        with _rings_lock:
            ring = _rings.get(device)
            if ring is None:
                ring = _rings[device] = _TableRing(device)
        key = (len(out_ptrs), n)
        nbytes = _table_bytes.get(key)
        if nbytes is None:
            nbytes = _table_bytes[key] = _lib.wsum_multi_table_bytes(*key)
        idx, h, d = ring.take(nbytes)
        try:
            _lib.wsum_multi_table_ptrs(code, ptrs, out_ptrs, numels, weights, h.data_ptr(), d.data_ptr(),
                                       int(s.cuda_stream), acc_in=acc_in)
        finally:
            ring.done(idx, s)
        return
    _lib.wsum_multi_ptrs(code, ptrs, out_ptrs, numels, weights, int(s.cuda_stream))


def wsum_sharded(peers: Sequence[torch.Tensor], weights: Sequence[float], devices: Sequence[torch.device],
                 out: Optional[torch.Tensor] = None, mode: str = "direct") -> torch.Tensor:
    """FedAvg of flat peers that may live on several GPUs of this process, bucket-sharded over
    ``devices`` (dla_wsum_sharded): shard s reduces bucket s of every peer on
    devices[s], reading the peers held by other GPUs over xGMI.  The result is bit-identical to
    ``wsum`` (each element keeps its list-order fold) and lands in ``out`` on devices[0].

    mode "direct": every shard writes its bucket straight into ``out`` (remote stores for the
    shards on other GPUs); "gather": every shard writes a buffer on its own GPU, then the buckets
    are copied into ``out`` peer-to-peer (gather=2).  Stream-ordered like any torch op: the
    shards wait for the peers' producers and ``out``'s device waits for every shard."""
    n = len(peers)
    if n < 1:
        raise IndexError("list index out of range")
    if len(weights) != n:
        raise AssertionError("len(weights) != len(peers)")
    devs = [torch.device(d) if not isinstance(d, torch.device) else d for d in devices]
    if not devs or any(d.type != "cuda" for d in devs):
        raise ValueError("wsum_sharded needs one or more HIP devices")
    require_device(devs[0])
    p0 = peers[0]
    code = dtype_code(p0.dtype)
    numel = p0.numel()
    for k, p in enumerate(peers):
        if p.device.type != "cuda" or not p.is_contiguous() or p.dtype != p0.dtype or p.numel() != numel:
            raise ValueError("peer %d must be a contiguous device tensor of %s x %d" % (k, p0.dtype, numel))
    if out is None:
        out = torch.empty(numel, dtype=p0.dtype, device=devs[0])
    if out.device != devs[0] or not out.is_contiguous() or out.numel() != numel or out.dtype != p0.dtype:
        raise ValueError("out must be a contiguous %s x %d tensor on %s" % (p0.dtype, numel, devs[0]))
    # the shards' streams wait for whatever produced the peers
    peer_devs = sorted({p.device.index for p in peers})
    shard_streams = [torch.cuda.current_stream(d) for d in devs]
    for pd in peer_devs:
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(pd))
        for st in shard_streams:
            st.wait_event(ev)
    if mode == "direct":
        outs, gather, keep = [out.data_ptr()] * len(devs), 0, []
    elif mode == "gather":
        keep = [out] + [torch.empty(numel, dtype=p0.dtype, device=d) for d in devs[1:]]
        outs, gather = [t.data_ptr() for t in keep], 2
    else:
        raise ValueError("mode must be 'direct' or 'gather'")
    _lib.wsum_sharded_ptrs(code, [d.index for d in devs], [p.data_ptr() for p in peers], weights, numel, outs,
                           gather, [int(st.cuda_stream) for st in shard_streams])
    # out's device waits for every shard's writes (direct) / its own copies (gather: already ordered)
    o_stream = shard_streams[0]
    done = []
    for st in shard_streams:
        ev = torch.cuda.Event()
        ev.record(st)
        done.append((st, ev))
        if st.cuda_stream != o_stream.cuda_stream:
            o_stream.wait_event(ev)
    # every peer-owning device's current stream waits for the shards that read its memory over
    # xGMI: the caching allocator reuses a freed peer (or a .contiguous() temporary of one) only for
    # later work on that stream, so a caller that drops the peers right after this call cannot have
    # their memory rewritten while a remote shard still reads it
    for pd in peer_devs:
        cur = torch.cuda.current_stream(pd)
        for st, ev in done:
            if st.cuda_stream != cur.cuda_stream:
                cur.wait_event(ev)
    for t, st in zip(keep[1:], shard_streams[1:]):
        t.record_stream(st)
        t.record_stream(o_stream)
    return out
