"""§8 f2 — the aggregator at the reference's call sites, on a light in-repo harness.

The reference's own integration tests need pyipv8's MockIPv8 (un-vendored, not
installable here).  Each test below restates only the aggregation-relevant lines of one
call site (cited) around this package's ModelManager / DeviceModelManager, and checks
the result bit-for-bit against the CPU oracle fed the same models, weights and order.
"""
import copy
import random
from math import floor
from types import SimpleNamespace

import pytest
import torch
from torch import nn

from oracle.fedavg_oracle import fedavg_param_lists, same_bits

pytestmark = pytest.mark.gpu


def _settings():
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod

    return SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG,
                           dfl=SimpleNamespace(sample_size=10, success_fraction=0.8))


class GNLeNetLike(nn.Module):
    """Parameter layout of the CIFAR-10 GNLeNet (configs[1]) plus a GroupNorm-free buffer."""

    def __init__(self, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        shapes = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,), (64, 32, 5, 5), (64,),
                  (64,), (64,), (10, 576), (10,)]
        self.ps = nn.ParameterList([nn.Parameter(torch.randn(s, generator=g) * 0.05) for s in shapes])
        self.register_buffer("steps", torch.tensor(seed))


def _expect(models, weights):
    return fedavg_param_lists([[p.detach().cpu().numpy() for p in m.parameters()] for m in models], weights, "f32")


def _check(result, models, weights):
    for p, want in zip(result.parameters(), _expect(models, weights)):
        assert same_bits(p.detach().cpu().numpy(), want, "f32")
    for b, b0 in zip(result.buffers(), models[0].buffers()):
        assert torch.equal(b.cpu(), b0.cpu())


@pytest.mark.parametrize("manager", ["ModelManager", "DeviceModelManager"])
def test_gl_gossip_merge(manager):
    """accdfl/gl/community.py:105-118: [self, remote] with age weights (None when the
    ages sum to 0), aggregate, reset, repeat."""
    from accdfl_amd.core import model_manager as mm_mod
    from accdfl_amd.core import wire

    local = GNLeNetLike(1)
    mm = getattr(mm_mod, manager)(local, _settings(), 0)
    my_age = 0
    for rnd, (remote_age, seed) in enumerate([(0, 11), (3, 12), (5, 13), (0, 14)]):
        incoming = GNLeNetLike(seed)
        detached = copy.deepcopy(mm.model)  # serialize/unserialize round trip (:108-109)
        mm.process_incoming_trained_model(b"me", detached)
        mm.process_incoming_trained_model(b"peer%d" % rnd, incoming)
        age_sum = remote_age + my_age
        weights = [my_age / age_sum, remote_age / age_sum] if age_sum > 0 else None
        my_age = max(remote_age, my_age)
        if manager == "DeviceModelManager":
            assert mm._uniform(), "both models staged into HBM on arrival: the slab path"
        result = mm.aggregate_trained_models(weights=weights)
        _check(result, [detached, incoming], weights or [0.5, 0.5])
        mm.model = result
        mm.reset_incoming_trained_models()
        my_age += 2  # "training" (:124)
        # the merged model travels on the wire in the reference's format
        assert set(wire.loads_state_dict(wire.serialize_model(result))) == set(result.state_dict())


def test_dl_round_assigns_registry_directly():
    """accdfl/dl/community.py:98-106: the registry is overwritten with a dict, every
    model is moved to the CPU, uniform weights."""
    from accdfl_amd.core.model_manager import DeviceModelManager

    mm = DeviceModelManager(GNLeNetLike(0), _settings(), 0)
    received = [(b"n%d" % i, GNLeNetLike(20 + i).to("cuda")) for i in range(5)]
    mm.incoming_trained_models = dict((x, y) for x, y in received)
    for pk in mm.incoming_trained_models.keys():
        mm.incoming_trained_models[pk] = mm.incoming_trained_models[pk].to(torch.device("cpu"))
    result = mm.aggregate_trained_models()
    _check(result, [m for _, m in received], [0.2] * 5)
    assert all(p.device.type == "cpu" for p in result.parameters())


def test_dl_round_staged_on_arrival():
    """accdfl/dl/community.py:98-106 with the models staged into HBM as they arrive: the receive handler
    also hands each (CPU) model to DeviceModelManager.process_incoming_trained_model; aggregate_models
    then runs the reference's own lines — the registry overwritten with a dict of the same models in the
    same order, each moved to the CPU (a no-op for CPU modules) — and the round reduces the staged slab
    rows (no H2D at aggregation), bit-exact, two rounds in a row."""
    from accdfl_amd.core.model_manager import DeviceModelManager

    mm = DeviceModelManager(GNLeNetLike(0), _settings(), 0, capacity=4)
    for rnd in range(2):
        incoming_models = []
        for i in range(5):  # on_receive: unserialized CPU models, staged as they arrive
            pk, model = b"n%d" % i, GNLeNetLike(20 + 10 * rnd + i)
            incoming_models.append((pk, model))
            mm.process_incoming_trained_model(pk, model)
        mm.incoming_trained_models = dict((x, y) for x, y in incoming_models)
        for pk in mm.incoming_trained_models.keys():
            mm.incoming_trained_models[pk] = mm.incoming_trained_models[pk].to(torch.device("cpu"))
        assert mm._uniform(), "the registry still holds exactly the staged rows"
        result = mm.aggregate_trained_models()
        _check(result, [m for _, m in incoming_models], [0.2] * 5)
        assert all(p.device.type == "cpu" for p in result.parameters())
        mm.model = result
        mm.reset_incoming_trained_models()


def test_staged_model_written_after_arrival_is_reread():
    """A model staged on arrival and then written in place (its version counter moves) no longer matches
    its slab row: the round averages the registry as it stands at aggregation time (fedavg.py:23-25)."""
    from accdfl_amd.core.model_manager import DeviceModelManager

    mm = DeviceModelManager(GNLeNetLike(0), _settings(), 0, capacity=3)
    models = [GNLeNetLike(60 + i) for i in range(3)]
    for i, m in enumerate(models):
        mm.process_incoming_trained_model(b"n%d" % i, m)
    assert mm._uniform()
    with torch.no_grad():
        models[1].ps[0].mul_(2.0)
    assert not mm._uniform()
    _check(mm.aggregate_trained_models(), models, [1 / 3.] * 3)


def test_dfl_aggregator_round_on_wire_bytes():
    """accdfl/dfl/community.py:606-689: one manager per round, models arrive (with a
    duplicate), the round completes at floor(sample_size * success_fraction) models,
    uniform average, the result is serialised for the next sample."""
    from accdfl_amd.core import wire
    from accdfl_amd.core.model_manager import DeviceModelManager

    settings = _settings()
    needed = floor(settings.dfl.sample_size * settings.dfl.success_fraction)
    peers = [GNLeNetLike(40 + i) for i in range(needed + 2)]
    arrivals = [(b"p%d" % i, wire.serialize_model(m)) for i, m in enumerate(peers)]
    arrivals.insert(3, arrivals[1])  # a retransmitted model: first arrival wins
    aggregations = {}
    sent = None
    for pk, data in arrivals:
        index = 7
        if index not in aggregations:
            aggregations[index] = DeviceModelManager(None, settings, 0, capacity=settings.dfl.sample_size,
                                                     template=GNLeNetLike(0))
        aggregations[index].process_incoming_serialized(pk, data)
        if len(aggregations[index].incoming_trained_models) >= needed:
            sent = aggregations[index].aggregate_serialized()
            break
    assert sent is not None
    got = wire.loads_state_dict(sent)
    want = _expect(peers[:needed], [float(1. / needed)] * needed)
    names = [n for n, _ in GNLeNetLike(0).named_parameters()]
    for name, w in zip(names, want):
        assert same_bits(got[name].numpy(), w, "f32"), name
    assert torch.equal(got["steps"], peers[0].steps)  # buffers from the first arrival


def test_simulation_evaluation_average_large_n():
    """simulations/gl/gl_simulation.py:96-105: up to 20 % of the network's models
    (here 26 of 128 nodes) averaged uniformly for evaluation."""
    from accdfl_amd.core.model_manager import ModelManager

    random.seed(0)
    nodes = [GNLeNetLike(100 + i) for i in range(128)]
    eligible = random.sample(list(enumerate(nodes)), min(len(nodes), int(len(nodes) * 0.2)))
    mm = ModelManager(None, _settings(), 0)
    for ind, model in eligible:
        mm.process_incoming_trained_model(b"%d" % ind, model)
    result = mm.aggregate_trained_models()
    n = len(eligible)
    _check(result, [m for _, m in eligible], [float(1. / n)] * n)
