"""Seeded random rounds through DeviceModelManager (the aggregator's registry with peers staged into
the HBM PeerSlab on arrival; accdfl/core/model_manager.py:39-58 + fedavg.py:13-26) against the C oracle.

Per case: a random template (1-5 parameters of one dtype, sometimes a 0-element one or a buffer, now
and then parameters of two dtypes, which the slab does not hold), a slab capacity that the round may
outgrow, 1-40 peers arriving as modules (host or device) or as serialize_model payloads (bytes, a
memoryview or EVA-style block lists), a duplicate arrival that must be ignored (:43-45), weights None
or random; two rounds per case.  aggregate_trained_models and aggregate_serialized are each checked
bit for bit (NaN as NaN) against fedavg.py over the registry's models in first-arrival order."""
import os
import numpy as np
import pytest
import torch
from torch import nn

import fuzz_cases as fz
from oracle.fedavg_oracle import same_bits

pytestmark = pytest.mark.gpu

# ACCDFL_AMD_FUZZ_SCALE=k runs k times the seeds (a long fuzz campaign; the suites keep the default)
N_CASES = 64 * int(os.environ.get("ACCDFL_AMD_FUZZ_SCALE", "1"))


class _Net(nn.Module):
    def __init__(self, params, buf=None):
        super().__init__()
        for i, p in enumerate(params):
            setattr(self, "p%d" % i, p)
        if buf is not None:
            self.register_buffer("stat", buf)


def _layout(rng):
    n_params = int(rng.integers(1, 6))
    numels = [int([1, 3, 64, 1000, 4097, 65_537, 250_001][rng.integers(7)]) for _ in range(n_params)]
    if rng.integers(0, 5) == 0:
        numels[int(rng.integers(n_params))] = 0
    dt = ["f32", "bf16", "f16"][rng.integers(3)]
    dts = [dt] * n_params
    if n_params > 1 and rng.integers(0, 6) == 0:
        dts[int(rng.integers(n_params))] = "f32" if dt != "f32" else "bf16"
    return [fz._shape_of(rng, m) for m in numels], dts, bool(rng.integers(0, 3) == 0)


def _model(rng, shapes, dts, buf, k, specials, tie=None):
    ps = [nn.Parameter(fz._values(rng, int(np.prod(s)) if s else 1, d, specials).view(s)) for s, d in zip(shapes, dts)]
    if tie is not None:  # one Parameter under two names: parameters() lists it once, state_dict() twice
        ps[tie[1]] = ps[tie[0]]
    return _Net(ps, torch.full((4,), float(k)) if buf else None)


def _blocks(rng, data: bytes):
    size = int([1, 17, 4096, 60_000, 1 << 20][rng.integers(5)])
    return [data[i:i + size] for i in range(0, len(data), size)]


def _check(out_params, want, desc):
    assert len(out_params) == len(want), desc
    for i, (p, (d, w)) in enumerate(zip(out_params, want)):
        assert fz.NAME[p.dtype] == d, "%s: parameter %d dtype" % (desc, i)
        assert same_bits(fz.bits(p), w, d), "%s: parameter %d" % (desc, i)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_device_model_manager_fuzz(seed):
    from types import SimpleNamespace

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager

    rng = np.random.default_rng(4000 + seed)
    shapes, dts, buf = _layout(rng)
    specials = rng.integers(0, 4) == 0
    trng = np.random.default_rng(seed + 77_777)  # ties drawn apart: the case's other draws are unchanged
    tie = tuple(sorted(int(x) for x in trng.choice(len(shapes), 2, replace=False))) \
        if len(shapes) > 1 and trng.integers(0, 5) == 0 else None
    template = _model(rng, shapes, dts, buf, -1, False, tie)
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0,
                            capacity=int(rng.integers(1, 9)), template=template)
    for rnd in range(2):
        n = int([1, 2, 3, 5, 8, 9, 16, 17, 40][rng.integers(9)])
        models = [_model(rng, shapes, dts, buf, k, specials, tie) for k in range(n)]
        how = []
        for k, m in enumerate(models):
            mode = int(rng.integers(0, 5))
            how.append(mode)
            key = b"peer%d" % k
            if mode == 0:
                mm.process_incoming_trained_model(key, m)
            elif mode == 1:
                mm.process_incoming_trained_model(key, m.to("cuda"))
                models[k] = m  # .to() moved the module in place: the registry holds the same object
            else:
                data = wire.serialize_model(m)
                payload = data if mode == 2 else memoryview(data) if mode == 3 else _blocks(rng, data)
                mm.process_incoming_serialized(key, payload)
            if k == 0 and rng.integers(0, 2):  # a re-send of peer 0 with other values: ignored
                mm.process_incoming_trained_model(key, _model(rng, shapes, dts, buf, 99, False, tie))
        weights = None if rng.integers(0, 3) == 0 else [float(x) for x in rng.dirichlet(np.ones(n))]
        want = fz.expected(models, weights)
        desc = "seed %d round %d: n=%d shapes=%s dtypes=%s arrivals=%s tie=%s" % (seed, rnd, n, shapes, sorted(set(dts)),
                                                                           how, tie)
        out = mm.aggregate_trained_models(weights)
        torch.cuda.synchronize()
        _check(list(out.parameters()), want, desc)
        if buf:
            assert torch.equal(out.stat.cpu(), torch.full((4,), 0.0)), desc  # models[0]'s buffer (:20)
        payload = mm.aggregate_serialized(weights)
        sd = wire.loads_state_dict(payload)
        names = [nm for nm, _ in out.named_parameters()]  # tied: the first name of each parameter
        _check([sd[nm] for nm in names], want, desc + " (aggregate_serialized)")
        if tie is not None:  # the alias carries the same average
            _check([sd["p%d" % tie[1]]], [want[names.index("p%d" % tie[0])]], desc + " (tied alias)")
        if buf:
            assert torch.equal(sd["stat"].cpu(), torch.full((4,), 0.0)), desc
        mm.reset_incoming_trained_models()
