"""Aggregation part of accdfl's ModelManager (accdfl/core/model_manager.py:20-58).

Only the aggregator-facing surface is rebuilt: the incoming-model registry
(:39-50), the aggregator selection (:52-54) and ``aggregate_trained_models`` (:56-58).
Training and evaluation (:60-114) are outside the hot path and not provided.

``DeviceModelManager`` is the MI355X-first variant: every received model is staged
into a device-resident PeerSlab the moment it arrives (the H2D copy overlaps the
wait for the remaining peers), so ``aggregate_trained_models`` is a single
device-resident reduce.  Registry semantics are identical: first arrival wins,
summation order = arrival order.
"""
from __future__ import annotations

import collections
import copy
import functools
import time
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
from accdfl_amd.core import wire
from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg, _center_copy


def _native_fingerprint(model: nn.Module) -> Optional[bytes]:
    """DeviceModelManager._fingerprint in native code (csrc/walk.cpp fingerprint: the same (identity,
    data pointer, version) of every parameter, as bytes), or None when the extension is absent or the
    model's tree holds a module class with its own parameter walk.  Classes not met before are classified
    once (fedavg._plain_walk), so a model gets the same kind of fingerprint at staging and at aggregation."""
    from accdfl_amd import _lib
    from accdfl_amd.core.gradient_aggregation import fedavg as _fa

    mod = _lib.walk_module()
    if mod is None or not hasattr(mod, "fingerprint"):
        return None
    fp = mod.fingerprint(model, _fa._PLAIN_SET)
    if fp is None:
        fresh = [type(sub) for sub in model.modules() if type(sub) not in _fa._plain_walk_cls]
        if any([_fa._plain_walk(cls) for cls in fresh]):
            fp = mod.fingerprint(model, _fa._PLAIN_SET)
    return fp


def _one_dtype(model: nn.Module) -> bool:
    """The model's parameters share one dtype (what a PeerSlab row holds)."""
    return len({p.dtype for p in model.parameters()}) == 1


class ModelManager:
    """Holds received peer models and aggregates them (model_manager.py:20-58)."""

    def __init__(self, model: Optional[nn.Module], settings, participant_index: int = 0):
        self.model: Optional[nn.Module] = model
        self.settings = settings
        self.participant_index: int = participant_index
        # Keeps track of the incoming trained models as aggregator (model_manager.py:39)
        self.incoming_trained_models: Dict[bytes, nn.Module] = {}

    def process_incoming_trained_model(self, peer_pk: bytes, incoming_model: nn.Module):
        if peer_pk in self.incoming_trained_models:
            # We already processed this model (model_manager.py:43-45)
            return
        self.incoming_trained_models[peer_pk] = incoming_model

    def reset_incoming_trained_models(self):
        self.incoming_trained_models = {}

    def get_aggregation_method(self):
        if self.settings.gradient_aggregation == GradientAggregationMethod.FEDAVG:
            return FedAvg

    def aggregate_trained_models(self, weights: List[float] = None) -> Optional[nn.Module]:
        models = [model for model in self.incoming_trained_models.values()]
        return self.get_aggregation_method().aggregate(models, weights=weights)


class WirePeer:
    """A peer model received as ``serialize_model`` bytes and decoded by
    ``wire.loads_state_dict``: its state dict, without the ``create_model`` +
    ``load_state_dict`` the reference runs (accdfl/core/models/__init__.py:13-16)."""

    def __init__(self, state_dict=None, make=None):
        """``state_dict``: the decoded tensors; or ``make``: a callable building them on first use (the
        native ingress path: the tensors over the page-locked ingress buffer are made only if the round
        reads them — models[0]'s buffers, or a fallback round)."""
        self._sd = state_dict
        self._make = make

    @property
    def state_dict(self):
        if self._sd is None:
            self._sd = self._make()
            self._make = None
        return self._sd

    def materialize(self, template: nn.Module) -> nn.Module:
        """The module the reference's ``unserialize_model`` would build."""
        m = copy.deepcopy(template)
        m.load_state_dict(self.state_dict)
        return m


class DeviceModelManager(ModelManager):
    """ModelManager whose received models are staged into HBM on arrival.

    ``capacity`` bounds the number of models one round holds (the DFL sample size, or
    1 + in-degree in DL); the slab grows if it is exceeded.  ``template`` is a module of
    the session's architecture (default: ``model``); it is needed only for models that
    arrive as wire bytes (``process_incoming_serialized``).
    """

    def __init__(self, model: Optional[nn.Module], settings, participant_index: int = 0, capacity: int = 8,
                 device: Optional[torch.device] = None, template: Optional[nn.Module] = None):
        super().__init__(model, settings, participant_index)
        self.template = template if template is not None else model
        from accdfl_amd.core.peer_slab import PeerSlab  # noqa: WPS433 (keeps import light for CPU-only users)

        self._slab_cls = PeerSlab
        self._capacity = capacity
        self._device = device
        self.slab: Optional["PeerSlab"] = None
        # what each slab row holds, in row order: (peer key, the registry entry, its parameters'
        # fingerprint at staging time) — the slab is used only while these still describe the
        # registry exactly (see _uniform)
        self._staged: List[tuple] = []
        # page-locked ingress buffers, one per registry position of a round (reused every round):
        # models that arrive as EVA block lists are gathered here instead of b''.join'ed
        self._ingress: List[Optional[torch.Tensor]] = []
        self._ingress_ev: List[Optional[torch.cuda.Event]] = []
        # next ingress slot of this round: only ever increases within a round (reset with the
        # registry), so a registry entry removed mid-round never hands its slot — still viewed by
        # a live WirePeer — to the next arrival
        self._ingress_next = 0
        # per-arrival phase record of process_incoming_serialized (None: off).  start_phases() turns it
        # on: decode + gather into the ingress buffer (CPU), the stage call (CPU) and HIP timing events
        # around each arrival's copies on the slab's copy stream (bench.py dfl_round's phase split)
        self.phases: Optional[dict] = None
        self._spec = None  # (template, parameter names, shapes): _row_spec's cache

    def start_phases(self) -> dict:
        self.phases = {"decode_gather_ms": [], "stage_issue_ms": [], "copy_events": []}
        return self.phases

    @staticmethod
    def _fingerprint(model) -> tuple:
        """Identity and in-place version of every parameter (torch bumps ``_version`` on each
        in-place write, so a model changed after it arrived no longer matches).  Writes through
        ``p.data`` (``p.data.copy_(...)``, ``p.data += ...``) bypass the version counter and are
        NOT detected: a caller that edits a registered model that way after it arrived must
        re-register it (or call ``reset_incoming_trained_models``)."""
        if isinstance(model, WirePeer):
            return ()
        fp = _native_fingerprint(model)
        if fp is not None:
            return fp
        return tuple((id(p), p.data_ptr(), p._version) for p in model.parameters())

    def process_incoming_trained_model(self, peer_pk: bytes, incoming_model: nn.Module):
        if peer_pk in self.incoming_trained_models:
            return
        self.incoming_trained_models[peer_pk] = incoming_model
        if self.slab is None:
            if not _one_dtype(incoming_model):
                return  # mixed-dtype model: the round falls back to FedAvg.aggregate (_uniform is False)
            self.slab = self._slab_cls.for_model(incoming_model, capacity=self._capacity, device=self._device)
        if self.slab.matches(list(incoming_model.parameters())) and len(self._staged) == self.slab.n:
            self.slab.stage(incoming_model)
            self._staged.append((peer_pk, incoming_model, self._fingerprint(incoming_model)))

    def _ingress_buffer(self, pos: int, nbytes: int) -> torch.Tensor:
        """Registry position ``pos``'s page-locked ingress buffer (grown to ``nbytes``), once the H2D that
        last read it has finished."""
        while len(self._ingress) <= pos:
            self._ingress.append(None)
            self._ingress_ev.append(None)
        ev = self._ingress_ev[pos]
        if ev is not None:
            ev.synchronize()
        buf = self._ingress[pos]
        if buf is None or buf.numel() < nbytes:
            buf = self._ingress[pos] = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        return buf

    def _ingress_alloc(self, pos: int, nbytes: int):
        """Bump allocator over registry position ``pos``'s page-locked ingress buffer (grown to
        ``nbytes``); waits until the H2D that last read that buffer has finished."""
        buf = self._ingress_buffer(pos, nbytes)
        off = [0]

        def alloc(n: int) -> torch.Tensor:
            a = off[0]
            off[0] = a + (n + 255) // 256 * 256
            if off[0] > buf.numel():
                raise ValueError("ingress buffer overflow")
            return buf[a:a + n]
        return alloc

    def _row_spec(self):
        """The template's parameter names and shapes in parameters() order (the slab row's layout),
        cached per template module."""
        if self._spec is None or self._spec[0] is not self.template:
            named = list(self.template.named_parameters())
            self._spec = (self.template, [n for n, _ in named], [tuple(p.shape) for _, p in named])
        return self._spec[1], self._spec[2]

    def process_incoming_serialized(self, peer_pk: bytes, data):
        """A model straight from the wire (§8 f1), decoded without executing the payload and
        staged into HBM, with no ``create_model`` / ``load_state_dict``.  ``data`` is the
        ``serialize_model`` payload as bytes, a memoryview (e.g. the model part of a DFL message,
        ``memoryview(result.data)[:model_data_len]``: no slice copy, accdfl/dfl/community.py:587)
        or the block list of the EVA transfer before its ``b''.join``
        (accdfl/util/eva/transfer/incoming.py:35; ``wire.split_blocks`` splits a DFL message's
        blocks).

        The payload is scanned natively (``wire.scan_state_dict``: the restricted opcode subset, no
        tensor built, no element byte copied); every storage is then gathered out of the payload into a
        page-locked ingress buffer by ONE batched memcpy, with the parameters back to back in
        ``parameters()`` order, so the peer's PeerSlab row goes to HBM as ONE asynchronous copy.  The
        peer's state dict (``WirePeer.state_dict``) is built over that buffer only if the round reads it.
        Payloads the native scan does not take (the extension absent, views, shared or mistyped
        parameter storages, anything outside a state dict's pickle) are decoded by the Python decoder
        as before; an unsafe payload is refused by it (``wire.UnsafePayloadError``).  The decoded
        tensors view the ingress buffer (or ``data``), which stays valid for this round (the buffer is
        reused one round later)."""
        if peer_pk in self.incoming_trained_models:
            return
        if self.template is None:
            raise ValueError("DeviceModelManager needs a template module to decode wire payloads")
        if not self.incoming_trained_models:
            self._ingress_next = 0  # a new round (also when the caller replaced the registry dict)
        if self.slab is None and _one_dtype(self.template):
            self.slab = self._slab_cls.for_model(self.template, capacity=self._capacity, device=self._device)
        ph = self.phases
        t0 = time.perf_counter() if ph is not None else 0.0
        lay = None
        if self.slab is not None and len(self._staged) == self.slab.n:
            names, shapes = self._row_spec()
            if shapes == self.slab.shapes:
                scan = wire.scan_state_dict(data)
                lay = scan.row_layout(names, self.slab.dtype, shapes) if scan is not None else None
        if lay is None:
            self._ingress_python(peer_pk, data, ph, t0)
            return
        offsets, total, row = lay
        pos = self._ingress_next
        self._ingress_next += 1
        buf = self._ingress_buffer(pos, total)[:total]
        scan.gather(buf, offsets)
        scan.release_payload()
        peer = WirePeer(make=functools.partial(scan.state_dict, buf, offsets))
        self.incoming_trained_models[peer_pk] = peer
        if ph is not None:
            t1 = time.perf_counter()
            ph["decode_gather_ms"].append((t1 - t0) * 1e3)
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(self.slab.copy_stream)
        self.slab.stage_flat(buf[:row].view(self.slab.dtype))
        self._staged.append((peer_pk, peer, ()))
        if ph is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(self.slab.copy_stream)
            ph["stage_issue_ms"].append((time.perf_counter() - t1) * 1e3)
            ph["copy_events"].append((e0, e1))
        ev = torch.cuda.Event()
        ev.record(self.slab.copy_stream)
        self._ingress_ev[pos] = ev

    def _ingress_python(self, peer_pk: bytes, data, ph, t0):
        """process_incoming_serialized through the Python decoder (wire.loads_state_dict): block lists
        gathered tensor by tensor into the ingress buffer, each parameter staged on its own."""
        alloc = None
        pos = -1
        if isinstance(data, (list, tuple)):
            pos = self._ingress_next
            self._ingress_next += 1
            n_tensors = len(self.template.state_dict())
            alloc = self._ingress_alloc(pos, sum(len(b) for b in data) + 256 * (n_tensors + 1))
        sd = wire.loads_state_dict(data, copy=False, alloc=alloc)  # views of `data` / the ingress buffer
        params = wire.parameter_tensors(sd, self.template)
        peer = WirePeer(sd)
        self.incoming_trained_models[peer_pk] = peer
        if ph is not None:
            t1 = time.perf_counter()
            ph["decode_gather_ms"].append((t1 - t0) * 1e3)
        if self.slab is None:
            return  # parameters of several dtypes: no slab; the round falls back to FedAvg.aggregate
        if ph is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(self.slab.copy_stream)
        if self.slab.matches(params) and len(self._staged) == self.slab.n:
            self.slab.stage(params)
            self._staged.append((peer_pk, peer, ()))
        if ph is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record(self.slab.copy_stream)
            ph["stage_issue_ms"].append((time.perf_counter() - t1) * 1e3)
            ph["copy_events"].append((e0, e1))
        if alloc is not None:
            ev = torch.cuda.Event()
            ev.record(self.slab.copy_stream)
            self._ingress_ev[pos] = ev

    def reset_incoming_trained_models(self):
        super().reset_incoming_trained_models()
        self._staged = []
        self._ingress_next = 0
        if self.slab is not None:
            self.slab.reset()

    def _modules(self) -> List[nn.Module]:
        return [m.materialize(self.template) if isinstance(m, WirePeer) else m
                for m in self.incoming_trained_models.values()]

    def _uniform(self) -> bool:
        """The slab's rows are exactly the registry's current entries, in order, unchanged since
        they were staged.  Otherwise (the registry was replaced or edited directly, as
        accdfl/dl/community.py:98-104 does, or a model was written in place after it arrived)
        the round is averaged from the registry itself, as the reference reads it at aggregate
        time (fedavg.py:23-25)."""
        items = list(self.incoming_trained_models.items())
        if self.slab is None or len(items) != self.slab.n or len(self._staged) != len(items):
            return False
        for (pk, m), (spk, sm, fp) in zip(items, self._staged):
            if pk != spk or m is not sm or self._fingerprint(m) != fp:
                return False
        return True

    def aggregate_trained_models(self, weights: List[float] = None) -> Optional[nn.Module]:
        if self.get_aggregation_method() is not FedAvg or not self._uniform():
            return self.get_aggregation_method().aggregate(self._modules(), weights=weights)
        entries = list(self.incoming_trained_models.values())
        n = len(entries)
        if not weights:
            weights = [float(1. / n) for _ in range(n)]
        else:
            assert len(weights) == n
        with torch.no_grad():
            first = entries[0]
            if isinstance(first, WirePeer):
                # deepcopy(models[0]) of the module unserialize_model would have built:
                # the template's structure with the first arrival's buffers.
                center = _center_copy(self.template)
                for name, buf in center.named_buffers():
                    if name in first.state_dict:
                        buf.copy_(first.state_dict[name])
            else:
                center = _center_copy(first)  # deepcopy(models[0]) minus the parameter values
            self.slab.reduce_into(list(center.parameters()), weights)
        return center

    def aggregate_serialized(self, weights: List[float] = None) -> bytes:
        """``serialize_model(aggregate_trained_models(weights))`` — the bytes a DFL
        aggregator sends back to the participants (accdfl/dfl/community.py:556-567).

        When the round's rows are staged (the slab is the registry), the averaged row is not
        copied into a result module first: the payload's parameter bytes come from HBM straight
        into the returned ``bytes`` (wire.DeviceSource), beside the buffers of the module
        ``aggregate_trained_models`` would have returned (models[0]'s, fedavg.py:20).  The
        encoded objects are the same."""
        if self.get_aggregation_method() is not FedAvg or not self._uniform():
            return wire.serialize_model(self.aggregate_trained_models(weights))
        entries = list(self.incoming_trained_models.values())
        n = len(entries)
        if not weights:
            weights = [float(1. / n) for _ in range(n)]
        else:
            assert len(weights) == n
        first = entries[0]
        # the module aggregate_trained_models returns: the template's structure with the first
        # arrival's buffers (wire peers), or deepcopy(models[0]) (module peers)
        structure = self.template if isinstance(first, WirePeer) else first
        params = list(structure.parameters())
        state = structure.state_dict(keep_vars=True)
        bufs = first.state_dict if isinstance(first, WirePeer) else state
        # every state-dict key of a parameter — a tied parameter is listed once by parameters() but
        # under each alias by state_dict() — maps to that parameter's averaged row, by identity
        offsets = {id(p): (o, p.shape) for p, o in zip(params, self.slab._offsets())}
        param_keys = {k for k, v in state.items() if id(v) in offsets}
        if (len(params) != len(self.slab.numels) or any(p.shape != s for p, s in zip(params, self.slab.shapes))
                or len(param_keys) < len(params)
                # the payload must carry what serialize_model(aggregate_trained_models()) carries: its
                # parameters are CPU tensors here (DeviceSource), so every other entry must be too
                or any(v.device.type != "cpu" for v in state.values())
                or any(bufs[k].device.type != "cpu" for k in state if k not in param_keys and k in bufs)):
            return wire.serialize_model(self.aggregate_trained_models(weights))
        with torch.no_grad():
            flat = self.slab._reduce_planned(weights)
            sd = collections.OrderedDict()
            for k, v in state.items():
                if k in param_keys:
                    off, shape = offsets[id(v)]
                    sd[k] = wire.DeviceSource(flat, off, shape)
                elif k in bufs and bufs[k].shape == v.shape:
                    # the round's models[0] buffers (deepcopy, fedavg.py:20), in the structure's dtype
                    sd[k] = bufs[k].detach().to(v.dtype)
                else:
                    sd[k] = v.detach()
            meta = getattr(state, "_metadata", None)
            if meta is not None:
                sd._metadata = meta
            return wire.dumps_state_dict(sd)
