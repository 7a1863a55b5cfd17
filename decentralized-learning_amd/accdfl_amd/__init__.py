"""accdfl_amd — MI355X-native gossip model aggregation for accdfl (devos50/decentralized-learning).

Only the aggregation hot path is rebuilt: the element-wise weighted
N-peer reduce behind accdfl's ``GradientAggregation.aggregate(models, weights)``
plugin API (reference: accdfl/core/gradient_aggregation/).  The reduce runs as a
hand-written gfx950 HIP kernel in ``libdlagg.so`` (C ABI: include/dlagg.h), driven
from Python on PyTorch-ROCm for device memory, streams and torch.distributed.

Import layout mirrors the reference package:
    accdfl_amd.core.gradient_aggregation            <- accdfl/core/gradient_aggregation/__init__.py
    accdfl_amd.core.gradient_aggregation.fedavg     <- accdfl/core/gradient_aggregation/fedavg.py
    accdfl_amd.core.model_manager                   <- accdfl/core/model_manager.py (aggregation part)
    accdfl_amd.core.peer_slab                       device staging of received peer models (HBM)
    accdfl_amd.core.sharding                        parameter-bucket sharding over ranks (RCCL)
"""

__version__ = "0.1.0"
