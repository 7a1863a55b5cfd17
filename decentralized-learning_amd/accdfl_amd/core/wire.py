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

import collections
import io
import pickle
from typing import Dict

import torch
from torch import nn


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


def _parse_storage_blob(blob) -> torch.TypedStorage:
    """Zero-copy decode of ``TypedStorage.__reduce__``'s blob (legacy torch.save of one
    storage; torch/serialization.py _legacy_save): the element data is viewed in place.
    ``blob`` may be bytes or a memoryview into the payload; only its small header is copied."""
    blob = memoryview(blob)
    f = io.BytesIO(bytes(blob[:65536]))  # the four header pickles are a few hundred bytes
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
    if pos + 8 > len(f.getbuffer()):
        raise UnsafePayloadError("storage blob header too long")
    n_saved = int.from_bytes(blob[pos:pos + 8], "little")
    start, nbytes = pos + 8, numel * esize
    if n_saved != numel or start + nbytes != len(blob):
        raise UnsafePayloadError("storage blob size mismatch")
    if numel == 0:
        data = torch.empty(0, dtype=dtype)
    else:
        import warnings

        with warnings.catch_warnings():  # read-only bytes: the tensor is never written in place
            warnings.simplefilter("ignore", UserWarning)
            data = torch.frombuffer(blob[start:start + nbytes], dtype=dtype)
    return torch.TypedStorage(wrap_storage=data.untyped_storage(), dtype=dtype, _internal=True)


def _load_storage_blob(blob: bytes):
    try:
        return _parse_storage_blob(blob)
    except UnsafePayloadError:
        raise
    except Exception:  # any other layout: torch's own safe loader
        return torch.load(io.BytesIO(blob), weights_only=True)


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


def _vm_loads(data) -> object:
    """A pickle VM for exactly the opcode subset ``pickle.dumps(state_dict)`` emits
    (protocols 2-4).  BINBYTES payloads come back as memoryviews into ``data``, so the
    nested storage blobs — i.e. all parameter bytes — are never copied; the only callables
    it can invoke are the three in ``_ALLOWED``."""
    mv = memoryview(data).cast("B")
    n = len(mv)
    pos = 0
    stack: list = []
    memo: dict = {}

    def take(k):
        nonlocal pos
        if pos + k > n:
            raise UnsafePayloadError("truncated payload")
        out = mv[pos:pos + k]
        pos += k
        return out

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

    while True:
        if pos >= n:
            raise UnsafePayloadError("truncated payload")
        op = mv[pos]
        pos += 1
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
            fn = _ALLOWED.get((module, name))
            if fn is None:
                raise UnsafePayloadError("accdfl_amd: refusing global %s.%s in a model payload" % (module, name))
            stack.append(_Global(fn))
        elif op == 0x63:      # GLOBAL (protocol <= 3)
            rest = bytes(mv[pos:pos + 256])
            module, name = rest.split(b"\n", 2)[:2]
            pos += len(module) + len(name) + 2
            fn = _ALLOWED.get((module.decode(), name.decode()))
            if fn is None:
                raise UnsafePayloadError("accdfl_amd: refusing global %s.%s in a model payload" % (
                    module.decode(errors="replace"), name.decode(errors="replace")))
            stack.append(_Global(fn))
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


def loads_state_dict(data: bytes, copy: bool = True) -> "collections.OrderedDict[str, torch.Tensor]":
    """Decode ``serialize_model`` bytes into the state dict (CPU tensors).

    The tensors' element data is parsed in place from the payload (no ``torch.load``
    pass, no copy of the parameter bytes: see ``_vm_loads``).  ``copy=True`` gives each tensor its own writable memory; ``copy=False``
    returns read-only views of the payload (what the ingress path stages to HBM)."""
    try:
        obj = _vm_loads(data)
    except _Unsupported:
        obj = _StateDictUnpickler(io.BytesIO(bytes(data))).load()
    if not isinstance(obj, dict) or not all(isinstance(k, str) and torch.is_tensor(v) for k, v in obj.items()):
        raise UnsafePayloadError("accdfl_amd: payload is not a state_dict")
    if copy:
        meta = getattr(obj, "_metadata", None)
        obj = collections.OrderedDict((k, v.clone()) for k, v in obj.items())
        if meta is not None:
            obj._metadata = meta
    return obj


def dumps_state_dict(state_dict: Dict[str, torch.Tensor]) -> bytes:
    """The reference's wire format for a state dict (accdfl/core/models/__init__.py:9-10)."""
    return pickle.dumps(state_dict)


def serialize_model(model: nn.Module) -> bytes:
    """accdfl/core/models/__init__.py:9-10: ``pickle.dumps(model.state_dict())``."""
    return dumps_state_dict(model.state_dict())


def parameter_tensors(state_dict: Dict[str, torch.Tensor], template: nn.Module):
    """The state dict's parameter tensors in ``template.parameters()`` order (the order
    fedavg.py:24 zips them in); raises KeyError if one is missing."""
    return [state_dict[name] for name, _ in template.named_parameters()]
