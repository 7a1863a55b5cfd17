"""§8 f1 at north-star scale: one DFL aggregator round of 8 peers x 25 M fp32 end to end, as
the reference's aggregator sees it (accdfl/dfl/community.py:576-673): every peer's message
arrives as EVA blocks (60 000-byte blocks, accdfl/core/session_settings.py:76), is split at
``model_data_len`` (:587-588) and decoded without the reference's b''.join
(accdfl/util/eva/transfer/incoming.py:35) into page-locked ingress buffers -> HBM PeerSlab;
the uniform average (:673) goes back out as serialize_model bytes (:556-567).  The decoded
result is compared bit for bit with the C oracle, over two rounds (the ingress buffers and
slab rows are reused).  Run on the MI355X: -m gpu."""
import pickle
from types import SimpleNamespace

import numpy as np
import pytest
import torch
from torch import nn

from c_oracle import c_wsum
from oracle.fedavg_oracle import same_bits

pytestmark = pytest.mark.gpu

N, P, BLOCK = 8, 25_000_000, 60_000


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from accdfl_amd import _lib

    assert _lib.lib().build_id == _lib.source_build_id()
    yield


def _message(k, seed):
    """A DFL 'trained_model' message: serialize_model bytes + the pickled population view."""
    from accdfl_amd.core import wire

    m = nn.Module()
    m.w = nn.Parameter(torch.randn(P, generator=torch.Generator().manual_seed(seed + k)) * 0.05)
    model_bytes = wire.serialize_model(m)
    view = pickle.dumps({"peer%d" % j: (j, seed) for j in range(5)})
    return m.w.detach().numpy().copy(), wire.payload_blocks(model_bytes + view, BLOCK), len(model_bytes)


def test_dfl_round_north_star_from_eva_blocks():
    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager

    template = nn.Module()
    template.w = nn.Parameter(torch.zeros(P))
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0,
                            capacity=N, template=template)
    for rnd, seed in enumerate((100, 900)):
        mm.reset_incoming_trained_models()
        flats = []
        for k in range(N):
            flat, blocks, model_len = _message(k, seed)
            flats.append(flat)
            head, tail = wire.split_blocks(blocks, model_len)
            assert pickle.loads(b"".join(tail))["peer0"] == (0, seed)
            mm.process_incoming_serialized(b"peer%d" % k, head)
        assert mm._uniform() and mm.slab.n == N
        out_bytes = mm.aggregate_serialized()  # uniform weights, as accdfl/dfl/community.py:673
        got = wire.loads_state_dict(out_bytes)["w"].numpy()
        want = c_wsum(flats, [float(1. / N)] * N, "f32")
        assert same_bits(got, want, "f32"), rnd
        assert pickle.loads(out_bytes)["w"].shape == (P,)  # the reference's own decoder reads it
