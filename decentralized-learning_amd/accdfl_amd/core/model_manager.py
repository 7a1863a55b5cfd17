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

from typing import Dict, List, Optional

import torch
import torch.nn as nn

from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg, _center_copy


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


class DeviceModelManager(ModelManager):
    """ModelManager whose received models are staged into HBM on arrival.

    ``capacity`` bounds the number of models one round holds (the DFL sample size, or
    1 + in-degree in DL); the slab grows if it is exceeded.
    """

    def __init__(self, model: Optional[nn.Module], settings, participant_index: int = 0, capacity: int = 8,
                 device: Optional[torch.device] = None):
        super().__init__(model, settings, participant_index)
        from accdfl_amd.core.peer_slab import PeerSlab  # noqa: WPS433 (keeps import light for CPU-only users)

        self._slab_cls = PeerSlab
        self._capacity = capacity
        self._device = device
        self.slab: Optional["PeerSlab"] = None

    def process_incoming_trained_model(self, peer_pk: bytes, incoming_model: nn.Module):
        if peer_pk in self.incoming_trained_models:
            return
        self.incoming_trained_models[peer_pk] = incoming_model
        try:
            if self.slab is None:
                self.slab = self._slab_cls.for_model(incoming_model, capacity=self._capacity, device=self._device)
            if self.slab.matches(list(incoming_model.parameters())):
                self.slab.stage(incoming_model)
        except TypeError:
            pass  # mixed-dtype model: the round falls back to FedAvg.aggregate (uniform_with is False)

    def reset_incoming_trained_models(self):
        super().reset_incoming_trained_models()
        if self.slab is not None:
            self.slab.reset()

    def aggregate_trained_models(self, weights: List[float] = None) -> Optional[nn.Module]:
        models = [model for model in self.incoming_trained_models.values()]
        if self.get_aggregation_method() is not FedAvg or self.slab is None or not self.slab.uniform_with(models):
            return super().aggregate_trained_models(weights)
        n = len(models)
        if not weights:
            weights = [float(1. / n) for _ in range(n)]
        else:
            assert len(weights) == n
        with torch.no_grad():
            center = _center_copy(models[0])  # deepcopy(models[0]) minus the parameter values
            self.slab.reduce_into(list(center.parameters()), weights)
        return center
