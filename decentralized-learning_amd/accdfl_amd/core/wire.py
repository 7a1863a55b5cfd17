"""accdfl's model wire format, decoded without executing the payload.

The reference serialises a model as ``pickle.dumps(model.state_dict())`` and decodes it
with ``create_model(...)`` + ``load_state_dict(pickle.loads(data))``
(accdfl/core/models/__init__.py:9-16).  Peers send these bytes over EVA
(accdfl/gl/community.py:105, accdfl/dfl/community.py:587-597), so ``pickle.loads`` runs
whatever the remote peer put in the payload.

``loads_state_dict`` accepts exactly what a ``state_dict`` pickle contains —
``collections.OrderedDict``, ``torch._utils._rebuild_tensor_v2`` and the nested
``torch.storage._load_from_bytes`` storage blobs, the latter decoded with
``torch.load(weights_only=True)`` — and refuses every other global.  It also skips
``create_model`` (a full model allocation + random init) and ``load_state_dict`` (a
second copy of every parameter): the tensors go straight to a PeerSlab row.

``dumps_state_dict`` / ``serialize_model`` produce the reference's exact format (plain
``pickle.dumps`` of the state dict), so averaged models travel back unchanged (f3).
"""
from __future__ import annotations

import bisect
import collections
import itertools
import io
import os
import pickle
import threading
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

import torch
from torch import nn

from accdfl_amd._lib import tuning_env as _tuning_env


class UnsafePayloadError(pickle.UnpicklingError):
    """The payload references something a state_dict pickle never contains."""


_LEGACY_MAGIC = 0x1950A86A20F9469CFC6C
_LEGACY_PROTOCOL = 1001
_STORAGE_DTYPES = {
    "FloatStorage": torch.float32, "DoubleStorage": torch.float64, "HalfStorage": torch.float16,
    "BFloat16Storage": torch.bfloat16, "LongStorage": torch.int64, "IntStorage": torch.int32,
    "ShortStorage": torch.int16, "CharStorage": torch.int8, "ByteStorage": torch.uint8,
    "BoolStorage": torch.bool,
}


class _BlobUnpickler(pickle.Unpickler):
    """The pickles inside one legacy ``torch.save`` storage blob: ints, a sys-info dict,
    the storage's persistent id (naming a ``torch.<X>Storage`` class) and the key list."""

    def find_class(self, module: str, name: str):
        if module == "torch" and name in _STORAGE_DTYPES:
            return ("storage_class", name)
        raise UnsafePayloadError("accdfl_amd: refusing global %s.%s in a storage blob" % (module, name))

    def persistent_load(self, pid):
        if (not isinstance(pid, tuple) or len(pid) != 6 or pid[0] != "storage" or not isinstance(pid[1], tuple)
                or pid[5] is not None):
            raise UnsafePayloadError("accdfl_amd: unexpected persistent id in a storage blob")
        return ("storage", _STORAGE_DTYPES[pid[1][1]], str(pid[2]), int(pid[4]))


class _Span:
    """A byte range of a block list (EVA's ``data_list``) that crosses block boundaries, kept
    as (host address, length) pieces of the blocks — int64 arrays, never joined unless asked.
    ``owner`` keeps the blocks alive."""
    __slots__ = ("addrs", "lens", "n", "owner", "_starts")

    def __init__(self, addrs: np.ndarray, lens: np.ndarray, owner):
        self.addrs = addrs
        self.lens = lens
        self.n = int(lens.sum())
        self.owner = owner
        self._starts = None

    def __len__(self):
        return self.n

    def sub(self, a: int, b: int):
        """(addresses, lengths) of the pieces covering [a, b) of this span, as int64 arrays
        (located by binary search: no per-piece Python work)."""
        if a >= b:
            return np.zeros(0, np.int64), np.zeros(0, np.int64)
        if self._starts is None:
            self._starts = np.concatenate(([0], np.cumsum(self.lens[:-1])))
        st = self._starts
        i = int(np.searchsorted(st, a, side="right")) - 1
        j = int(np.searchsorted(st, b - 1, side="right")) - 1
        addrs = self.addrs[i:j + 1].copy()
        lens = self.lens[i:j + 1].copy()
        lens[-1] = b - st[j]
        d = a - st[i]
        addrs[0] += d
        lens[0] -= d
        return addrs, lens

    def read(self, a: int, b: int) -> bytes:
        import ctypes

        return b"".join(ctypes.string_at(int(q), int(ln)) for q, ln in zip(*self.sub(a, b)))


_BYTES_DATA = bytes.__basicsize__ - 1  # CPython: offset of a bytes object's payload


def _check_bytes_layout() -> bool:
    import ctypes

    probe = b"accdfl-amd-probe"
    return ctypes.string_at(id(probe) + _BYTES_DATA, len(probe)) == probe


_BYTES_ADDR_OK = _check_bytes_layout()


def _block_address(block) -> int:
    """Host address of a block's first byte (no copy): bytes objects from the object itself,
    other buffers through numpy."""
    if type(block) is bytes and _BYTES_ADDR_OK:
        return id(block) + _BYTES_DATA
    return np.frombuffer(block, dtype=np.uint8).__array_interface__["data"][0]


# A 100 MB model is ~1 700 EVA blocks: the per-block bookkeeping (addresses, lengths) comes from one
# native call (csrc/walk.cpp block_table, a few ns per block) or, without the extension, from C-level
# map operations; round 3 spent 0.5-0.65 ms per 100 MB peer in Python loops over the blocks (bench.py
# dfl_round phases, profiles/r04a).

def _block_table(blocks: list) -> Tuple[np.ndarray, np.ndarray]:
    """(addresses, byte lengths) of every block, as int64 arrays."""
    from accdfl_amd import _lib

    mod = _lib.walk_module()
    if mod is not None:
        return mod.block_table(blocks)
    lens = np.fromiter(map(len, blocks), dtype=np.int64, count=len(blocks))
    if _BYTES_ADDR_OK:
        addrs = np.fromiter(map(id, blocks), dtype=np.int64, count=len(blocks))
        addrs += _BYTES_DATA
    else:
        addrs = np.zeros(len(blocks), dtype=np.int64)
    if not _BYTES_ADDR_OK or set(map(type, blocks)) != {bytes}:
        for i, b in enumerate(blocks):
            if type(b) is not bytes or not _BYTES_ADDR_OK:
                addrs[i] = _block_address(b)
                lens[i] = memoryview(b).nbytes
    return addrs, lens


# Gathers into a page-locked ingress buffer (read next by the H2D DMA, not by the CPU) use streaming
# stores (dla_host_copy_batch_ex, DLA_COPY_STREAMING); ACCDFL_AMD_INGRESS_NT=0 turns them off (A/B).
_INGRESS_NT = _tuning_env("ACCDFL_AMD_INGRESS_NT", "1") != "0"


# When a list, _gather appends each gather's wall time in ms (bench.py dfl_round's phase split).
GATHER_MS: Optional[list] = None


def _gather(addrs, lens, dst: torch.Tensor) -> None:
    """Copy the pieces back to back into the host uint8 tensor ``dst`` (one native batched
    memcpy, threaded from 4 MiB: libdlagg's dla_host_copy_batch)."""
    from accdfl_amd import _lib

    if not len(lens):
        return
    t0 = time.perf_counter() if GATHER_MS is not None else 0.0
    dsts = np.empty(len(lens), dtype=np.int64)
    dsts[0] = dst.data_ptr()
    np.cumsum(lens[:-1], out=dsts[1:])
    dsts[1:] += dsts[0]
    _lib.host_copy_batch(dsts, addrs, lens, streaming=_INGRESS_NT and int(lens.sum()) >= (4 << 20) and dst.is_pinned())
    if GATHER_MS is not None:
        GATHER_MS.append((time.perf_counter() - t0) * 1e3)


def _parse_storage_blob(blob, alloc=None) -> torch.TypedStorage:
    """Zero-copy decode of ``TypedStorage.__reduce__``'s blob (legacy torch.save of one
    storage; torch/serialization.py _legacy_save): the element data is viewed in place.
    ``blob`` may be bytes, a memoryview into the payload, or a _Span of a block list; only its
    small header is copied.  A _Span's element bytes are gathered into ``alloc(nbytes)`` (a host
    uint8 tensor, e.g. a page-locked ingress buffer) when given, else joined."""
    span = blob if isinstance(blob, _Span) else None
    if span is None:
        blob = memoryview(blob)
        head = bytes(blob[:65536])
    else:
        head = span.read(0, min(65536, len(span)))
    f = io.BytesIO(head)  # the four header pickles are a few hundred bytes
    u = _BlobUnpickler(f)
    if u.load() != _LEGACY_MAGIC or u.load() != _LEGACY_PROTOCOL:
        raise UnsafePayloadError("not a legacy storage blob")
    info = u.load()
    if not isinstance(info, dict) or not info.get("little_endian", False):
        raise UnsafePayloadError("unsupported storage blob byte order")
    u = _BlobUnpickler(f)
    obj = u.load()
    keys = _BlobUnpickler(f).load()
    if not (isinstance(obj, tuple) and obj[0] == "storage" and keys == [obj[2]]):
        raise UnsafePayloadError("storage blob does not hold exactly one storage")
    _, dtype, _, numel = obj
    pos = f.tell()
    esize = torch.empty((), dtype=dtype).element_size()
    if pos + 8 > len(head):
        raise UnsafePayloadError("storage blob header too long")
    n_saved = int.from_bytes(head[pos:pos + 8], "little")
    start, nbytes = pos + 8, numel * esize
    if n_saved != numel or start + nbytes != len(blob):
        raise UnsafePayloadError("storage blob size mismatch")
    if numel == 0:
        data = torch.empty(0, dtype=dtype)
    elif span is not None:
        if alloc is not None:
            dst = alloc(nbytes)
            _gather(*span.sub(start, start + nbytes), dst)
            # the storage must START at dst: dst is a slice of a larger buffer (the ingress bump
            # allocator), whose untyped_storage() is the whole buffer — the tensor rebuilt on it
            # (_rebuild_tensor_v2, offset 0) would read the buffer's first bytes.  A storage slice
            # aliases dst's bytes and keeps the buffer alive.
            a = dst.storage_offset()
            return torch.TypedStorage(wrap_storage=dst.untyped_storage()[a:a + nbytes], dtype=dtype, _internal=True)
        else:
            data = torch.frombuffer(bytearray(span.read(start, start + nbytes)), dtype=dtype)
    else:
        import warnings

        with warnings.catch_warnings():  # read-only bytes: the tensor is never written in place
            warnings.simplefilter("ignore", UserWarning)
            data = torch.frombuffer(blob[start:start + nbytes], dtype=dtype)
    return torch.TypedStorage(wrap_storage=data.untyped_storage(), dtype=dtype, _internal=True)


_LEGACY_HEAD = pickle.dumps(_LEGACY_MAGIC, protocol=2)[:4]  # PROTO 2, LONG1 of 10 bytes: a legacy blob's start


def _load_storage_blob(blob, alloc=None):
    try:
        return _parse_storage_blob(blob, alloc)
    except UnsafePayloadError:
        raise
    except Exception:  # any other layout (the zipfile format): torch's own safe loader
        if isinstance(blob, _Span):
            blob = blob.read(0, len(blob))
        if bytes(memoryview(blob)[:4]) == _LEGACY_HEAD:
            # a legacy blob the parser refused (its sizes disagree): torch's legacy loader would allocate
            # the element count the header claims, whatever the blob holds
            raise UnsafePayloadError("accdfl_amd: malformed legacy storage blob")
        return torch.load(io.BytesIO(blob), weights_only=True)


def _check_lengths(flat: bytes) -> None:
    """Every length an opcode of the pickle claims (BINBYTES8, BYTEARRAY8, BINUNICODE8, FRAME, ...) fits in
    the bytes that follow it — checked before the restricted unpickler runs, since CPython's unpickler
    allocates a claimed length before it reads (a few corrupt bytes must not make the decoder allocate
    gigabytes).  pickletools.genops reads each argument and stops at the first that runs past the end."""
    import pickletools

    try:
        for _ in pickletools.genops(flat):
            pass
    except Exception as e:
        raise UnsafePayloadError("accdfl_amd: malformed model payload (%s)" % str(e)[:200])


_ALLOWED = {
    ("collections", "OrderedDict"): collections.OrderedDict,
    ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
    ("torch.storage", "_load_from_bytes"): _load_storage_blob,
}


class _StateDictUnpickler(pickle.Unpickler):
    def find_class(self, module: str, name: str):
        try:
            return _ALLOWED[(module, name)]
        except KeyError:
            raise UnsafePayloadError("accdfl_amd: refusing global %s.%s in a model payload" % (module, name))


class _Unsupported(Exception):
    """An opcode outside the state_dict subset: hand the payload to the restricted unpickler."""


class _Global:
    __slots__ = ("fn",)

    def __init__(self, fn):
        self.fn = fn


_MARK = object()


class _BlockReader:
    """Sequential reads over a list of byte blocks (EVA's ``data_list``, before its
    ``b''.join``, accdfl/util/eva/transfer/incoming.py:35): a read inside one block is a
    memoryview into it, a short read across blocks is joined, a long one is a _Span.  A 100 MB
    model is ~1 700 blocks: the blocks are located by bisection over their start offsets and
    a long read's pieces are list slices, so no Python code runs per block."""

    def __init__(self, blocks):
        blocks = blocks if type(blocks) is list else list(blocks)
        addrs, lens = _block_table(blocks)
        if len(lens) and not lens.all():  # drop empty blocks
            keep = np.flatnonzero(lens)
            blocks = [blocks[i] for i in keep.tolist()]
            addrs, lens = addrs[keep], lens[keep]
        self.blocks = blocks
        self.addrs, self.lens_np = addrs, lens
        self.lens = lens.tolist()
        self.starts = [0] + np.cumsum(lens[:-1]).tolist() if len(lens) else []
        self.views = [None] * len(self.blocks)
        self.pos = 0
        self.n = int(lens.sum())
        # the block the last read ended in: (its view, its start, its end) — most reads (the pickle's
        # opcodes and their arguments) fall inside it and skip the bisection
        self.cur = (b"", 0, 0)

    @property
    def left(self) -> int:
        return self.n - self.pos

    def _view(self, i: int) -> memoryview:
        v = self.views[i]
        if v is None:
            v = self.views[i] = memoryview(self.blocks[i]).cast("B")
        return v

    def take(self, k: int):
        a = self.pos
        b = a + k
        v, s0, e0 = self.cur
        if s0 <= a and b <= e0:  # inside the current block
            self.pos = b
            return v[a - s0:b - s0]
        if k > self.n - a:
            raise UnsafePayloadError("truncated payload")
        self.pos = b
        if k == 0:
            return b""
        st, lens = self.starts, self.lens
        i = bisect.bisect_right(st, a) - 1
        o = a - st[i]
        if o + k <= lens[i]:
            v = self._view(i)
            self.cur = (v, st[i], st[i] + lens[i])
            return v[o:o + k]
        j = bisect.bisect_right(st, b - 1) - 1
        self.cur = (self._view(j), st[j], st[j] + lens[j])  # the next read starts in block j (or after it)
        if k <= 4096:  # a short read across a block boundary: joined
            pieces = [self._view(i)[o:]]
            pieces += [self._view(q) for q in range(i + 1, j)]
            pieces.append(self._view(j)[:b - st[j]])
            return b"".join(pieces)
        addrs = self.addrs[i:j + 1].copy()
        out_lens = self.lens_np[i:j + 1].copy()
        addrs[0] += o
        out_lens[0] -= o
        out_lens[-1] = b - st[j]
        return _Span(addrs, out_lens, self.blocks)


def _vm_loads(data, alloc: Optional[Callable[[int], torch.Tensor]] = None) -> object:
    """A pickle VM for exactly the opcode subset ``pickle.dumps(state_dict)`` emits
    (protocols 2-4).  BINBYTES payloads come back as memoryviews into ``data``, so the
    nested storage blobs — i.e. all parameter bytes — are never copied; the only callables
    it can invoke are the three in ``_ALLOWED``.  ``data`` may also be a list of blocks (an EVA
    transfer's ``data_list``): storage bytes that cross blocks are then gathered into
    ``alloc(nbytes)`` (a host uint8 tensor) in place of the reference's full ``b''.join``."""
    if isinstance(data, (list, tuple)):
        rd = _BlockReader(data)
        n = rd.left

        def take(k):
            return rd.take(k)
    else:
        mv = memoryview(data).cast("B")
        n = len(mv)
        rd = None

        def take(k):
            nonlocal pos
            if pos + k > n:
                raise UnsafePayloadError("truncated payload")
            out = mv[pos:pos + k]
            pos += k
            return out
    pos = 0
    stack: list = []
    memo: dict = {}
    storage_loader = _Global(_load_storage_blob if alloc is None else
                             (lambda blob: _load_storage_blob(blob, alloc)))

    def u(k):
        return int.from_bytes(take(k), "little")

    def pop_mark():
        i = len(stack) - 1
        while i >= 0 and stack[i] is not _MARK:
            i -= 1
        if i < 0:
            raise UnsafePayloadError("pickle: missing MARK")
        items = stack[i + 1:]
        del stack[i:]
        return items

    def allowed(module, name):
        fn = _ALLOWED.get((module, name))
        if fn is None:
            raise UnsafePayloadError("accdfl_amd: refusing global %s.%s in a model payload" % (module, name))
        return storage_loader if fn is _load_storage_blob else _Global(fn)

    while True:
        if rd is None:
            if pos >= n:
                raise UnsafePayloadError("truncated payload")
            op = mv[pos]
            pos += 1
        else:
            op = take(1)[0]
        if op == 0x80:        # PROTO
            if u(1) > 4:
                raise _Unsupported()
        elif op == 0x95:      # FRAME (length only: frames are inline)
            take(8)
        elif op == 0x2E:      # STOP
            if len(stack) != 1:
                raise UnsafePayloadError("pickle: bad stack at STOP")
            return stack[0]
        elif op == 0x28:      # MARK
            stack.append(_MARK)
        elif op == 0x8C:      # SHORT_BINUNICODE
            stack.append(str(take(u(1)), "utf-8"))
        elif op == 0x58:      # BINUNICODE
            stack.append(str(take(u(4)), "utf-8"))
        elif op == 0x8D:      # BINUNICODE8
            stack.append(str(take(u(8)), "utf-8"))
        elif op == 0x94:      # MEMOIZE
            memo[len(memo)] = stack[-1]
        elif op == 0x71:      # BINPUT
            memo[u(1)] = stack[-1]
        elif op == 0x72:      # LONG_BINPUT
            memo[u(4)] = stack[-1]
        elif op == 0x68:      # BINGET
            stack.append(memo[u(1)])
        elif op == 0x6A:      # LONG_BINGET
            stack.append(memo[u(4)])
        elif op == 0x93:      # STACK_GLOBAL
            name = stack.pop()
            module = stack.pop()
            stack.append(allowed(module, name))
        elif op == 0x63:      # GLOBAL (protocol <= 3)
            if rd is not None:
                raise _Unsupported()
            rest = bytes(mv[pos:pos + 256])
            module, name = rest.split(b"\n", 2)[:2]
            pos += len(module) + len(name) + 2
            stack.append(allowed(module.decode(errors="replace"), name.decode(errors="replace")))
        elif op == 0x29:      # EMPTY_TUPLE
            stack.append(())
        elif op == 0x85:      # TUPLE1
            stack[-1:] = [(stack[-1],)]
        elif op == 0x86:      # TUPLE2
            stack[-2:] = [tuple(stack[-2:])]
        elif op == 0x87:      # TUPLE3
            stack[-3:] = [tuple(stack[-3:])]
        elif op == 0x74:      # TUPLE
            stack.append(tuple(pop_mark()))
        elif op == 0x52:      # REDUCE
            args = stack.pop()
            fn = stack.pop()
            if not isinstance(fn, _Global) or not isinstance(args, tuple):
                raise UnsafePayloadError("pickle: REDUCE on a non-allowed callable")
            stack.append(fn.fn(*args))
        elif op == 0x4A:      # BININT
            stack.append(int.from_bytes(take(4), "little", signed=True))
        elif op == 0x4B:      # BININT1
            stack.append(u(1))
        elif op == 0x4D:      # BININT2
            stack.append(u(2))
        elif op == 0x8A:      # LONG1
            stack.append(int.from_bytes(take(u(1)), "little", signed=True))
        elif op == 0x4E:      # NONE
            stack.append(None)
        elif op == 0x88:      # NEWTRUE
            stack.append(True)
        elif op == 0x89:      # NEWFALSE
            stack.append(False)
        elif op == 0x7D:      # EMPTY_DICT
            stack.append({})
        elif op == 0x5D:      # EMPTY_LIST
            stack.append([])
        elif op == 0x61:      # APPEND
            v = stack.pop()
            stack[-1].append(v)
        elif op == 0x65:      # APPENDS
            items = pop_mark()
            stack[-1].extend(items)
        elif op == 0x73:      # SETITEM
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif op == 0x75:      # SETITEMS
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items) - 1, 2):
                d[items[i]] = items[i + 1]
        elif op == 0x62:      # BUILD: only OrderedDict instance attributes (state_dict._metadata)
            state = stack.pop()
            inst = stack[-1]
            if not isinstance(inst, collections.OrderedDict) or not isinstance(state, dict) or \
                    set(state) - {"_metadata"}:
                raise UnsafePayloadError("pickle: BUILD outside a state_dict's _metadata")
            for k, v in state.items():
                setattr(inst, k, v)
        elif op == 0x42:      # BINBYTES: a view into the payload, not a copy
            stack.append(take(u(4)))
        elif op == 0x43:      # SHORT_BINBYTES
            stack.append(take(u(1)))
        elif op == 0x8E:      # BINBYTES8
            stack.append(take(u(8)))
        elif op == 0x47:      # BINFLOAT
            import struct

            stack.append(struct.unpack(">d", take(8))[0])
        else:
            raise _Unsupported()


def loads_state_dict(data, copy: bool = True, alloc: Optional[Callable[[int], torch.Tensor]] = None
                     ) -> "collections.OrderedDict[str, torch.Tensor]":
    """Decode ``serialize_model`` bytes into the state dict (CPU tensors).

    ``data``: the payload as bytes / a memoryview (e.g. the model part of a DFL message,
    ``memoryview(result.data)[:model_data_len]``, accdfl/dfl/community.py:587, without the
    reference's slice copy), or the list of blocks an EVA transfer received, before the
    reference's ``b''.join(data_list)`` (accdfl/util/eva/transfer/incoming.py:35).
    The tensors' element data is parsed in place from the payload (no ``torch.load``
    pass, no copy of the parameter bytes: see ``_vm_loads``); a tensor whose bytes cross
    EVA blocks is gathered into ``alloc(nbytes)`` (a host uint8 tensor; a page-locked ingress
    buffer on the staging path) or, without ``alloc``, joined for that tensor alone.
    ``copy=True`` gives each tensor its own writable memory; ``copy=False`` returns views (what
    the ingress path stages to HBM)."""
    try:
        obj = _vm_loads(data, alloc)
    except _Unsupported:
        flat = b"".join(memoryview(b) for b in data) if isinstance(data, (list, tuple)) else bytes(data)
        _check_lengths(flat)
        obj = _StateDictUnpickler(io.BytesIO(flat)).load()
    if not isinstance(obj, dict) or not all(isinstance(k, str) and torch.is_tensor(v) for k, v in obj.items()):
        raise UnsafePayloadError("accdfl_amd: payload is not a state_dict")
    if copy:
        meta = getattr(obj, "_metadata", None)
        clones = collections.OrderedDict((k, v.clone()) for k, v in obj.items())
        storages = [v.untyped_storage().data_ptr() for v in obj.values() if v.numel()]
        # a clone is exact only for a tensor that is the whole of its own storage: same strides, offset 0,
        # and the storage no larger than the tensor (pickle.loads keeps a view's storage and offset), and
        # listed once (pickle.loads keeps one object under both keys, empty tensors included)
        if len(set(storages)) == len(storages) and len({id(v) for v in obj.values()}) == len(obj) and all(
                c.numel() == 0 or (c.stride() == v.stride() and v.storage_offset() == 0
                                   and v.untyped_storage().nbytes() == v.numel() * v.element_size())
                for c, v in zip(clones.values(), obj.values())):
            obj = clones  # every tensor dense and on a storage of its own: a clone is what pickle.loads gives
        else:
            # entries sharing a storage (tied weights) or strided views: keep both as pickle.loads does
            # (deepcopy copies each storage once and rebuilds every view on it)
            import copy as _copy

            del clones
            obj = _copy.deepcopy(collections.OrderedDict(obj))
        if meta is not None:
            obj._metadata = meta
    return obj


class StateDictScan:
    """A ``serialize_model`` payload scanned in native code (csrc/walk.cpp ``scan_state_dict``: the same
    restricted opcode subset and allow-list as ``_vm_loads``, run over the block list in place, no tensor
    built and no element byte copied).  ``entries`` maps each state-dict key to its description
    ``(tag, storage index, storage offset, sizes, strides, requires_grad)`` — tied entries share one
    description object — and ``storages`` lists ``(dtype name, numel, payload position, nbytes)``.

    ``gather(buf, offsets)`` copies every storage's bytes out of the payload into ``buf`` (a host uint8
    tensor; storage i at byte ``offsets[i]``) with one batched memcpy; ``state_dict(buf, offsets)`` then
    makes the tensors over ``buf`` — one storage per pickled storage, as pickle.loads gives."""

    __slots__ = ("entries", "storages", "addrs", "lens", "owner")

    def __init__(self, entries, storages, addrs, lens, owner):
        self.entries, self.storages, self.addrs, self.lens, self.owner = entries, storages, addrs, lens, owner

    def gather(self, buf: torch.Tensor, offsets: np.ndarray) -> None:
        from accdfl_amd import _lib

        if not self.storages:
            return
        t0 = time.perf_counter() if GATHER_MS is not None else 0.0
        st = np.asarray([(p, n) for _, _, p, n in self.storages], dtype=np.int64).reshape(-1, 2)
        offsets = np.asarray(offsets, dtype=np.int64)
        if len(offsets) != len(st) or (offsets < 0).any() or int((offsets + st[:, 1]).max()) > buf.numel() \
                or buf.dtype != torch.uint8 or buf.device.type != "cpu" or not buf.is_contiguous():
            raise ValueError("StateDictScan.gather: offsets outside the buffer")
        dst = offsets + buf.data_ptr()
        d, s, n = _lib.walk_module().span_pieces(self.addrs, self.lens, np.ascontiguousarray(st[:, 0]),
                                                 np.ascontiguousarray(st[:, 1]), dst)
        if len(n):
            _lib.host_copy_batch(d, s, n, streaming=_INGRESS_NT and int(n.sum()) >= (4 << 20) and buf.is_pinned())
        if GATHER_MS is not None:
            GATHER_MS.append((time.perf_counter() - t0) * 1e3)

    def release_payload(self) -> None:
        """Forget the payload's blocks once gathered (the state dict is built from the buffer alone)."""
        self.addrs = self.lens = self.owner = None

    def state_dict(self, buf: torch.Tensor, offsets: np.ndarray) -> "collections.OrderedDict[str, torch.Tensor]":
        from accdfl_amd import _lib

        return _lib.walk_module().build_state_dict(buf, offsets.astype(np.int64), self.entries, self.storages,
                                                   collections.OrderedDict)

    def row_layout(self, names: Sequence[str], dtype: torch.dtype, shapes: Sequence[tuple], native: bool = True):
        """Where a PeerSlab row's parameters can come from in one piece: when the entries ``names``
        (``template.named_parameters()`` order) are dense tensors of ``dtype`` and ``shapes``, each the
        whole of a storage of its own, ``(offsets, total bytes, row bytes)`` — a byte offset per storage
        that puts those parameters back to back from byte 0 (the row the slab stages with ONE copy), every
        other storage after them, 256-byte aligned.  None otherwise (a missing key, a view, a shared or
        mis-typed storage): the caller decodes through the general path."""
        dname = str(dtype).replace("torch.", "")
        from accdfl_amd import _lib

        mod = _lib.walk_module()
        if native and hasattr(mod, "row_layout"):  # csrc/walk.cpp: the same rules, no Python frame per parameter
            return mod.row_layout(self.entries, self.storages, names if type(names) is list else list(names), dname,
                                  shapes if type(shapes) is list else [tuple(s) for s in shapes])
        offsets = np.full(len(self.storages), -1, dtype=np.int64)
        off = 0
        for name, shape in zip(names, shapes):
            d = self.entries.get(name)
            if d is None:
                return None
            _, sidx, soff, size, stride, _ = d
            sdt, numel, _, nbytes = self.storages[sidx]
            if soff != 0 or size != shape or sdt != dname or offsets[sidx] >= 0:
                return None
            n = 1
            for s in size:
                n *= s
            if numel != n or stride != _contiguous_strides(size):
                return None
            offsets[sidx] = off
            off += nbytes
        row = off
        off = -(-off // 256) * 256
        for i, (_, _, _, nbytes) in enumerate(self.storages):
            if offsets[i] < 0:
                offsets[i] = off
                off += -(-nbytes // 256) * 256
        return offsets, max(off, 1), row


def _contiguous_strides(size) -> tuple:
    st, acc = [], 1
    for s in reversed(size):
        st.append(acc)
        acc *= s
    return tuple(reversed(st))


def scan_state_dict(data) -> Optional[StateDictScan]:
    """``data`` (bytes, a memoryview or an EVA block list) scanned natively, or None when the native
    extension is absent or the payload holds anything outside a state dict's pickle (the Python decoder
    then decodes it or refuses it with its own error)."""
    from accdfl_amd import _lib

    mod = _lib.walk_module()
    if mod is None or not hasattr(mod, "scan_state_dict"):
        return None
    blocks = list(data) if isinstance(data, (list, tuple)) else [data]
    addrs, lens = _block_table(blocks)
    if len(lens) and not lens.all():
        keep = np.flatnonzero(lens)
        addrs, lens = addrs[keep], lens[keep]
    res = mod.scan_state_dict(np.ascontiguousarray(addrs), np.ascontiguousarray(lens), collections.OrderedDict)
    if res is None:
        return None
    return StateDictScan(res[0], res[1], addrs, lens, blocks)


_STORAGE_NAMES = {v: k for k, v in _STORAGE_DTYPES.items()}
_SENTINEL_BYTES = 1 << 16   # >= the pickler's 64 KiB frame target: written outside any frame


class _StorageRef:
    """Pickles as ``torch.storage._load_from_bytes(<sentinel>)``: a placeholder the fast path
    replaces by the storage's legacy blob."""

    def __init__(self, token: bytes):
        self.token = token

    def __reduce__(self):
        return (torch.storage._load_from_bytes, (self.token,))


class _TensorRef:
    """Pickles like a contiguous CPU tensor that owns its storage (torch.Tensor.__reduce_ex__:
    ``_rebuild_tensor_v2(storage, 0, size, stride, False, OrderedDict())``)."""

    def __init__(self, t: torch.Tensor, token: bytes):
        self.size, self.stride, self.token = tuple(t.size()), tuple(t.stride()), token

    def __reduce__(self):
        return (torch._utils._rebuild_tensor_v2,
                (_StorageRef(self.token), 0, self.size, self.stride, False, collections.OrderedDict()))


class _PidPickler(pickle.Pickler):
    def persistent_id(self, obj):
        return obj if isinstance(obj, tuple) and obj and obj[0] == "storage" else None


def _legacy_blob_header(t: torch.Tensor, key: str) -> bytes:
    """Everything of a legacy ``torch.save(storage)`` blob (torch/serialization.py
    _legacy_save, what TypedStorage.__reduce__ embeds) before the storage's raw bytes: magic,
    protocol, sys info, the storage's persistent id, the key list, the element count."""
    f = io.BytesIO()
    for obj in (_LEGACY_MAGIC, _LEGACY_PROTOCOL,
                dict(protocol_version=_LEGACY_PROTOCOL, little_endian=True,
                     type_sizes=dict(short=2, int=4, long=4))):
        pickle.dump(obj, f, protocol=2)
    _PidPickler(f, protocol=2).dump(("storage", getattr(torch, _STORAGE_NAMES[t.dtype]), key, "cpu", t.numel(),
                                     None))
    pickle.dump([key], f, protocol=2)
    f.write(t.numel().to_bytes(8, "little"))
    return f.getvalue()


def _owns_storage(t: torch.Tensor) -> bool:
    return (t.device.type == "cpu" and t.is_contiguous() and t.storage_offset() == 0
            and t.numel() * t.element_size() == t.untyped_storage().nbytes() and t.dtype in _STORAGE_NAMES
            and not t.requires_grad)


class DeviceSource:
    """A state-dict entry whose values live in HBM: ``numel`` elements of ``flat`` (a contiguous device
    tensor of the entry's dtype) from element ``offset`` on, with the entry's ``shape``.  dumps_state_dict
    encodes it like the CPU tensor it stands for and copies its bytes from the device straight into
    the returned payload (egress without the result module: accdfl/dfl/community.py:556-567)."""

    def __init__(self, flat: torch.Tensor, offset: int, shape):
        self.flat, self.offset, self.shape = flat, offset, tuple(shape)
        self.numel = 1
        for d in self.shape:
            self.numel *= d
        self.dtype = flat.dtype
        self._meta = None

    @property
    def meta(self) -> torch.Tensor:
        """What _TensorRef / _legacy_blob_header read: sizes, contiguous strides, dtype, numel (made only
        when a payload layout is first encoded)."""
        if self._meta is None:
            self._meta = torch.empty(self.shape, dtype=self.dtype, device="meta")
        return self._meta

    def data_ptr(self) -> int:
        return self.flat.data_ptr() + self.offset * self.flat.element_size()

    def nbytes(self) -> int:
        return self.numel * self.flat.element_size()

    def to_cpu(self) -> torch.Tensor:
        return self.flat[self.offset:self.offset + self.numel].view(self.shape).cpu()


def dumps_state_dict(state_dict: Dict[str, torch.Tensor]) -> bytes:
    """The reference's wire format for a state dict (accdfl/core/models/__init__.py:9-10: a
    pickle of the OrderedDict whose tensors reduce to ``_rebuild_tensor_v2`` over
    ``_load_from_bytes`` legacy storage blobs), decodable by the reference's own
    ``pickle.loads`` + ``load_state_dict``.

    ``pickle.dumps`` copies a large tensor's bytes three times (the legacy torch.save into a
    BytesIO, its getvalue, the pickler's output), 42 ms for a 25 M fp32 model.  Here each
    tensor of >= 64 KiB that owns its storage is pickled as a 64 KiB placeholder, written
    outside any pickle frame, which is then replaced by the storage's blob header and its raw
    bytes: the parameter bytes are copied once, into the returned bytes.  The objects encoded
    are the same as ``pickle.dumps``'s; the bytes differ only in framing and memo layout (the
    reference's own bytes are not reproducible anyway: storage keys are memory addresses).

    Round 6: a state dict whose every tensor owns its storage (a module's state_dict(); the
    DeviceSources of aggregate_serialized) is written from a cached template of its LAYOUT
    (_PayloadTemplate: the pickle and every storage blob's header made once per layout), so a round
    costs one batched memcpy of the tensors' bytes (and one chunked D2H for the entries in HBM), not a
    pickle pass and a torch.save header per tensor (16 google_speech ResNet-34 models, 218 entries:
    aggregate_serialized 15.6 ms in profiles/r06b, ~10 of them per-tensor pickling)."""
    if _BYTES_ADDR_OK:
        plan = _template_plan(state_dict)
        if plan is not None:
            return plan[0].fill(plan[1])
    big = []
    skeleton = collections.OrderedDict()
    refs = {}  # id(entry) -> its placeholder: an entry listed twice pickles once, as pickle.dumps memoizes it
    for k, v in state_dict.items():
        if id(v) in refs:
            skeleton[k] = refs[id(v)]
        elif isinstance(v, DeviceSource):
            if v.nbytes() >= _SENTINEL_BYTES and _BYTES_ADDR_OK:
                token = os.urandom(_SENTINEL_BYTES)
                skeleton[k] = refs[id(v)] = _TensorRef(v.meta, token)
                big.append((token, v))
            else:
                # small: through the CPU like any tensor, once (an entry listed twice stays one tensor)
                skeleton[k] = refs[id(v)] = v.to_cpu()
        elif torch.is_tensor(v) and v.numel() * v.element_size() >= _SENTINEL_BYTES and _owns_storage(v):
            token = os.urandom(_SENTINEL_BYTES)
            skeleton[k] = refs[id(v)] = _TensorRef(v, token)
            big.append((token, v))
        else:
            skeleton[k] = v
    meta = getattr(state_dict, "_metadata", None)
    if meta is not None:
        skeleton._metadata = meta
    skel = pickle.dumps(skeleton)
    if not big:
        return skel
    # (address, length, keep-alive) of every piece of the output, in order; a DeviceSource's piece
    # is a device address, copied by _join_pieces from HBM
    pieces, pos = [], 0
    skel_addr = id(skel) + _BYTES_DATA
    for i, (token, t) in enumerate(big):
        at = skel.find(token, pos)
        if at < 5 or skel[at - 5] != 0x42 or int.from_bytes(skel[at - 4:at], "little") != _SENTINEL_BYTES:
            return pickle.dumps(_cpu_state_dict(state_dict))  # unexpected pickler output: the stock path
        pieces.append((skel_addr + pos, at - 5 - pos, skel))
        dev = isinstance(t, DeviceSource)
        head = _legacy_blob_header(t.meta if dev else t, str(i))
        nbytes = t.nbytes() if dev else t.numel() * t.element_size()
        n = len(head) + nbytes
        head = (b"B" + n.to_bytes(4, "little") if n < 1 << 32 else b"\x8e" + n.to_bytes(8, "little")) + head
        pieces.append((id(head) + _BYTES_DATA, len(head), head))
        pieces.append((t.data_ptr(), nbytes, t))
        pos = at + _SENTINEL_BYTES
    pieces.append((skel_addr + pos, len(skel) - pos, skel))
    return _join_pieces(pieces)


class _PayloadTemplate:
    """dumps_state_dict's bytes for one state-dict layout — keys, each entry's dtype and shape, which
    entries are one tensor, ``_metadata`` — with the tensors' raw bytes left out: ``gaps[i]`` (the
    pickle's own bytes and the next storage blob's header, one bytes object) come before slot i, which
    holds distinct tensor i's ``slots[i]`` raw bytes; ``gaps[-1]`` ends the payload.  Built once per layout
    by pickling 64 KiB tokens in place of the tensors (what dumps_state_dict's general path splices)."""

    __slots__ = ("gaps", "slots", "gap_off", "slot_off", "total")

    def __init__(self, state_dict, sources):
        base = os.urandom(_SENTINEL_BYTES)
        tokens = [i.to_bytes(8, "little") + base[8:] for i in range(len(sources))]
        refs = {id(v): _TensorRef(v.meta if isinstance(v, DeviceSource) else v, tok) for v, tok in zip(sources, tokens)}
        skeleton = collections.OrderedDict((k, refs[id(v)]) for k, v in state_dict.items())
        meta = getattr(state_dict, "_metadata", None)
        if meta is not None:
            skeleton._metadata = meta
        skel = pickle.dumps(skeleton)
        gaps, slots, pos = [], [], 0
        for i, (tok, v) in enumerate(zip(tokens, sources)):
            at = skel.find(tok, pos)
            if at < 5 or skel[at - 5] != 0x42 or int.from_bytes(skel[at - 4:at], "little") != _SENTINEL_BYTES:
                raise ValueError("unexpected pickler output")
            dev = isinstance(v, DeviceSource)
            head = _legacy_blob_header(v.meta if dev else v, str(i))
            nbytes = v.nbytes() if dev else v.numel() * v.element_size()
            n = len(head) + nbytes
            op = b"B" + n.to_bytes(4, "little") if n < 1 << 32 else b"\x8e" + n.to_bytes(8, "little")
            gaps.append(skel[pos:at - 5] + op + head)
            slots.append(nbytes)
            pos = at + _SENTINEL_BYTES
        gaps.append(skel[pos:])
        self.gaps, self.slots = gaps, slots
        self.gap_off, self.slot_off, o = [], [], 0
        for g, n in zip(gaps, slots + [0]):
            self.gap_off.append(o)
            o += len(g)
            self.slot_off.append(o)
            o += n
        self.slot_off.pop()
        self.total = o

    def fill(self, sources) -> bytes:
        """The payload with ``sources`` (CPU tensors / DeviceSources, in slot order) in the slots."""
        from accdfl_amd import _lib

        out = _new_bytes(None, self.total)
        base = id(out) + _BYTES_DATA
        dst, src, ln, dev = [], [], [], []
        for g, o in zip(self.gaps, self.gap_off):
            if g:
                dst.append(base + o)
                src.append(id(g) + _BYTES_DATA)
                ln.append(len(g))
        for v, o, n in zip(sources, self.slot_off, self.slots):
            if not n:
                continue
            if isinstance(v, DeviceSource) and v.flat.device.type != "cpu":
                dev.append((base + o, v))
            else:  # a CPU tensor, or a DeviceSource over a CPU row
                dst.append(base + o)
                src.append(v.data_ptr())
                ln.append(n)
        _lib.host_copy_batch(dst, src, ln)
        if dev:
            _copy_device_segments(dev)
        return out


_TEMPLATES: "collections.OrderedDict[tuple, _PayloadTemplate]" = collections.OrderedDict()
_TEMPLATES_KEPT = 8
_templates_lock = threading.Lock()


def _template_plan(state_dict):
    """(the cached _PayloadTemplate of ``state_dict``'s layout, its distinct tensors in slot order), or
    None when an entry is not a tensor that owns its storage or a DeviceSource (views, requires_grad,
    other objects: the general path encodes those)."""
    sig, sources, first = [], [], {}
    for k, v in state_dict.items():
        j = first.get(id(v))
        if j is not None:
            sig.append((k, j))
            continue
        if isinstance(v, DeviceSource):
            sig.append((k, v.dtype, v.shape))
        elif torch.is_tensor(v) and _owns_storage(v):
            sig.append((k, v.dtype, tuple(v.shape)))
        else:
            return None
        first[id(v)] = len(sources)
        sources.append(v)
    if not sources:
        return None
    meta = getattr(state_dict, "_metadata", None)
    key = (type(state_dict), tuple(sig), None if meta is None else pickle.dumps(meta))
    with _templates_lock:
        tpl = _TEMPLATES.get(key)
        if tpl is not None:
            _TEMPLATES.move_to_end(key)
    if tpl is None:
        try:
            tpl = _PayloadTemplate(state_dict, sources)
        except ValueError:
            return None
        with _templates_lock:
            _TEMPLATES[key] = tpl
            while len(_TEMPLATES) > _TEMPLATES_KEPT:
                _TEMPLATES.popitem(last=False)
    return tpl, sources


def _copy_device_segments(segs) -> None:
    """Each (host address, DeviceSource) of ``segs``: the source's bytes from HBM into host memory at the
    address (a fresh payload: pageable, not yet faulted in).  Per device tensor the sources live on, the
    byte range they span is copied D2H in chunks through the two page-locked bounce buffers on a side
    stream, and each chunk's pieces are copied out by ONE threaded batched memcpy while the next chunk's
    D2H runs (_copy_from_device for many sources at once: one D2H stream per round, not one per tensor)."""
    groups: Dict[int, list] = {}
    for addr, v in segs:
        groups.setdefault(id(v.flat), []).append((addr, v))
    for items in groups.values():
        flat = items[0][1].flat
        es = flat.element_size()
        dst = np.array([a for a, _ in items], dtype=np.int64)
        off = np.array([v.offset * es for _, v in items], dtype=np.int64)
        n = np.array([v.nbytes() for _, v in items], dtype=np.int64)
        dev = flat.device
        with _egress_lock:
            st = _egress_bounce.get(dev)
            if st is None:
                st = _egress_bounce[dev] = (
                    [torch.empty(_EGRESS_CHUNK, dtype=torch.uint8, pin_memory=True) for _ in range(2)],
                    torch.cuda.Stream(dev), [None, None], threading.Lock())
        bufs, stream, evs, lock = st
        with lock:
            _copy_segment_chunks(flat, dst, off, n, bufs, stream, evs)


def _copy_segment_chunks(flat, dst, off, n, bufs, stream, evs):
    from accdfl_amd import _lib

    lo, hi = int(off.min()), int((off + n).max())
    stream.wait_stream(torch.cuda.current_stream(flat.device))  # the reduce that produced flat is done
    flat_u8 = flat.view(torch.uint8)
    chunks = [(a, min(_EGRESS_CHUNK, hi - a)) for a in range(lo, hi, _EGRESS_CHUNK)]

    def issue(c):
        a, ln = chunks[c]
        with torch.cuda.stream(stream):
            bufs[c & 1][:ln].copy_(flat_u8[a:a + ln], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        evs[c & 1] = ev

    issue(0)
    for c in range(len(chunks)):
        if c + 1 < len(chunks):
            issue(c + 1)
        evs[c & 1].synchronize()
        a, ln = chunks[c]
        s = np.maximum(off, a)
        e = np.minimum(off + n, a + ln)
        m = s < e
        if m.any():
            _lib.host_copy_batch(dst[m] + (s[m] - off[m]), bufs[c & 1].data_ptr() + (s[m] - a), e[m] - s[m],
                                 streaming=_EGRESS_NT)


def _cpu_state_dict(state_dict):
    out = collections.OrderedDict((k, v.to_cpu() if isinstance(v, DeviceSource) else v) for k, v in state_dict.items())
    meta = getattr(state_dict, "_metadata", None)
    if meta is not None:
        out._metadata = meta
    return out


def _join_pieces(pieces) -> bytes:
    """One ``bytes`` holding the pieces back to back.  The object is created uninitialised
    (PyBytes_FromStringAndSize(NULL, n), as CPython's own builders do) and filled by libdlagg's
    threaded batched memcpy before any other code can see it, so a 100 MB model's page faults
    and copy are spread over threads instead of b''.join's one.  Pieces that are DeviceSources
    come from HBM through _copy_from_device."""
    import ctypes

    total = sum(ln for _, ln, _ in pieces)
    has_dev = any(isinstance(k, DeviceSource) for _, _, k in pieces)
    if not has_dev and (not _BYTES_ADDR_OK or total < (8 << 20)):
        return b"".join(ctypes.string_at(a, ln) if ln else b"" for a, ln, _ in pieces)
    from accdfl_amd import _lib

    out = _new_bytes(None, total)
    dsts = list(itertools.accumulate([ln for _, ln, _ in pieces[:-1]], initial=id(out) + _BYTES_DATA))
    host = [(d, a, ln) for d, (a, ln, k) in zip(dsts, pieces) if ln and not isinstance(k, DeviceSource)]
    if host:
        _lib.host_copy_batch([d for d, _, _ in host], [a for _, a, _ in host], [ln for _, _, ln in host])
    for d, (a, ln, k) in zip(dsts, pieces):
        if ln and isinstance(k, DeviceSource):
            _copy_from_device(d, k, ln)
    return out


# Bounce chunk of _copy_from_device (its copy-out runs on up to 8 threads from 16 MiB: a chunk of
# 8 MiB gets only 4) and the store kind of the copy-out (A/B knobs).
_EGRESS_CHUNK = int(float(_tuning_env("ACCDFL_AMD_EGRESS_CHUNK_MB", "32")) * (1 << 20))
_EGRESS_NT = _tuning_env("ACCDFL_AMD_EGRESS_NT", "0") == "1"
_egress_bounce = {}
_egress_lock = threading.Lock()


def _copy_from_device(dst: int, src: "DeviceSource", nbytes: int) -> None:
    """``nbytes`` from HBM at ``src`` into host memory at ``dst`` (a fresh payload: pageable, not
    yet faulted in): chunked D2H into two page-locked bounce buffers on a side stream, each chunk
    copied out by the threaded batched memcpy (which spreads the destination's page faults over
    threads) while the next chunk's D2H runs.  A D2H straight into the fresh pageable payload would
    fault it in on one thread (11-13 ms per 100 MB on the MI355X hosts, core/host_memory.py)."""
    dev = src.flat.device
    with _egress_lock:
        st = _egress_bounce.get(dev)
        if st is None:
            st = _egress_bounce[dev] = (
                [torch.empty(_EGRESS_CHUNK, dtype=torch.uint8, pin_memory=True) for _ in range(2)],
                torch.cuda.Stream(dev), [None, None], threading.Lock())
    bufs, stream, evs, lock = st
    with lock:  # one copy-out at a time per device: the bounce buffers are shared
        _copy_chunks(dst, src, nbytes, bufs, stream, evs)


def _copy_chunks(dst, src, nbytes, bufs, stream, evs):
    from accdfl_amd import _lib

    dev = src.flat.device
    stream.wait_stream(torch.cuda.current_stream(dev))  # the reduce that produced src is done
    flat_u8 = src.flat.view(torch.uint8)
    base = src.offset * src.flat.element_size()
    chunks = [(a, min(_EGRESS_CHUNK, nbytes - a)) for a in range(0, nbytes, _EGRESS_CHUNK)]

    def issue(c):
        a, ln = chunks[c]
        with torch.cuda.stream(stream):
            bufs[c & 1][:ln].copy_(flat_u8[base + a:base + a + ln], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        evs[c & 1] = ev

    issue(0)
    for c in range(len(chunks)):
        if c + 1 < len(chunks):
            issue(c + 1)
        evs[c & 1].synchronize()
        a, ln = chunks[c]
        _lib.host_copy_batch([dst + a], [bufs[c & 1].data_ptr()], [ln], streaming=_EGRESS_NT)


def _bytes_builder():
    import ctypes

    fn = ctypes.pythonapi.PyBytes_FromStringAndSize
    fn.restype = ctypes.py_object
    fn.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
    return fn


_new_bytes = _bytes_builder()


def serialize_model(model: nn.Module) -> bytes:
    """accdfl/core/models/__init__.py:9-10: ``pickle.dumps(model.state_dict())`` (the same
    objects, large tensors written with one copy: see dumps_state_dict)."""
    return dumps_state_dict(model.state_dict())


def parameter_tensors(state_dict: Dict[str, torch.Tensor], template: nn.Module):
    """The state dict's parameter tensors in ``template.parameters()`` order (the order
    fedavg.py:24 zips them in); raises KeyError if one is missing."""
    return [state_dict[name] for name, _ in template.named_parameters()]


def split_blocks(blocks: Sequence, n: int):
    """(the first n bytes, the rest) of a block list, as two block lists — the DFL message split
    at ``model_data_len`` (accdfl/dfl/community.py:587-588) with no copy: blocks that fall
    wholly on one side are passed through as they are (so a ``bytes`` block keeps its cheap
    address), the block holding byte n becomes two memoryview slices."""
    blocks = blocks if type(blocks) is list else list(blocks)
    if n <= 0:
        return [], blocks
    lens = _block_table(blocks)[1]
    ends = np.cumsum(lens)
    total = int(ends[-1]) if len(ends) else 0
    if total < n:
        raise ValueError("split_blocks: the blocks hold %d bytes, fewer than %d" % (total, n))
    k = int(np.searchsorted(ends, n))  # the first block that ends at or past byte n
    if int(ends[k]) == n:
        return blocks[:k + 1], blocks[k + 1:]
    start = int(ends[k] - lens[k])
    v = memoryview(blocks[k]).cast("B")
    return blocks[:k] + [v[:n - start]], [v[n - start:]] + blocks[k + 1:]


def payload_blocks(data: bytes, block_size: int) -> List[bytes]:
    """``data`` cut into ``block_size`` blocks, as an EVA transfer delivers them
    (accdfl/util/eva/transfer/outgoing.py:37-40 ``_get_block``: one ``block_size`` slice per
    data packet)."""
    return [data[i:i + block_size] for i in range(0, len(data), block_size)]
