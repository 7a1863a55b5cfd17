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


def _parse_storage_blob(blob: bytes) -> torch.TypedStorage:
    """Zero-copy decode of ``TypedStorage.__reduce__``'s blob (legacy torch.save of one
    storage; torch/serialization.py _legacy_save): the element data is viewed in place."""
    f = io.BytesIO(blob)
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
            data = torch.frombuffer(memoryview(blob)[start:start + nbytes], dtype=dtype)
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


def loads_state_dict(data: bytes, copy: bool = True) -> "collections.OrderedDict[str, torch.Tensor]":
    """Decode ``serialize_model`` bytes into the state dict (CPU tensors).

    The tensors' element data is parsed in place from the payload (no ``torch.load``
    pass).  ``copy=True`` gives each tensor its own writable memory; ``copy=False``
    returns read-only views of the payload (what the ingress path stages to HBM)."""
    obj = _StateDictUnpickler(io.BytesIO(data)).load()
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
