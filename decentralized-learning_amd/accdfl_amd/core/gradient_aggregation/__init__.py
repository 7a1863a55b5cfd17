"""Aggregator plugin contract — mirrors accdfl/core/gradient_aggregation/__init__.py:1-17.

Same names, same staticmethod signature, same enum value: a session whose settings
say ``gradient_aggregation = GradientAggregationMethod.FEDAVG`` (=1,
accdfl/core/session_settings.py:73) selects this package's HIP FedAvg.
"""
from abc import abstractmethod
from enum import IntEnum
from typing import List

from torch import nn


class GradientAggregationMethod(IntEnum):
    FEDAVG = 1


class GradientAggregation:

    @staticmethod
    @abstractmethod
    def aggregate(models: List[nn.Module], weights: List[float]):
        pass
