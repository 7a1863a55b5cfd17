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


def _load_storage_blob(blob: bytes):
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


def loads_state_dict(data: bytes) -> "collections.OrderedDict[str, torch.Tensor]":
    """Decode ``serialize_model`` bytes into the state dict (CPU tensors)."""
    obj = _StateDictUnpickler(io.BytesIO(data)).load()
    if not isinstance(obj, dict) or not all(isinstance(k, str) and torch.is_tensor(v) for k, v in obj.items()):
        raise UnsafePayloadError("accdfl_amd: payload is not a state_dict")
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
