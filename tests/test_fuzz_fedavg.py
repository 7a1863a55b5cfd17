"""Seeded random rounds through FedAvg.aggregate against the C oracle (tests/fuzz_cases.py: peer
counts, shapes, strides, dtypes and their mixes, zip truncation, weight forms and IEEE specials drawn
from one seed per case), bit for bit with NaN compared as NaN.

The CPU test checks the two restatements of the reference against each other on every case (the C
oracle and oracle/fedavg_oracle.py's numpy port); the GPU tests run each case through the product on
CPU-resident and on device-resident models and also check that the result keeps models[0]'s
dtypes, shapes, strides, device, requires_grad and buffers and that no input changed."""
import numpy as np
import pytest
import torch

import fuzz_cases as fz
from oracle.fedavg_oracle import fedavg_bits, fedavg_bits_mixed, same_bits

SEEDS = list(range(fz.N_CASES))
_VIEW = {"f32": np.float32, "f64": np.float64, "f16": np.float16, "bf16": np.uint16}


def _port_expected(models, weights):
    n = len(models)
    w = [float(1. / n) for _ in range(n)] if not weights else [float(x) for x in weights]
    plist = [list(m.parameters()) for m in models]
    out = []
    for i in range(len(plist[0])):
        ks = [k for k in range(n) if len(plist[k]) > i]
        dts = [fz.NAME[plist[k][i].dtype] for k in ks]
        flats = [fz.bits(plist[k][i]).view(_VIEW[d]) for k, d in zip(ks, dts)]
        if len(set(dts)) == 1:
            res = fedavg_bits(flats, [w[k] for k in ks], dts[0])
        else:
            res = fedavg_bits_mixed(flats, dts, [w[k] for k in ks])
        out.append((dts[0], np.asarray(res).reshape(-1)))
    return out


@pytest.mark.parametrize("seed", SEEDS)
def test_c_oracle_matches_numpy_port_on_fuzz_case(seed):
    models, weights, desc = fz.make_case(seed)
    for i, ((d1, a), (d2, b)) in enumerate(zip(fz.expected(models, weights), _port_expected(models, weights))):
        assert d1 == d2
        assert same_bits(a, b, d1), "%s: parameter %d, C oracle vs numpy port" % (desc, i)


def test_fuzz_cases_cover_the_contract():
    """The generator reaches every feature it claims (so a change to it cannot silently narrow the
    fuzz): each dtype, mixed rounds, truncation, empty models, transposed views, 0-element and
    0-d parameters, two-pass peer counts, every weight form, specials and buffers."""
    seen = set()
    for seed in SEEDS:
        models, weights, desc = fz.make_case(seed)
        params = [p for m in models for p in m.parameters()]
        seen.update(fz.NAME[p.dtype] for p in params)
        if len({(i, p.dtype) for m in models for i, p in enumerate(m.parameters())}) > \
                len({i for m in models for i, _ in enumerate(m.parameters())}):
            seen.add("mixed")
        lens = [len(list(m.parameters())) for m in models]
        if len(set(lens)) > 1:
            seen.add("truncation")
        if 0 in lens:
            seen.add("empty model")
        if any(not p.is_contiguous() for p in params):
            seen.add("transposed")
        if any(p.numel() == 0 for p in params):
            seen.add("0 elements")
        if any(p.dim() == 0 for p in params):
            seen.add("0-d")
        if len(models) > 128:
            seen.add("two passes")
        seen.add("weights=" + desc.split("weights=")[1].split(" specials=")[0])
        if "tie=None" not in desc:
            seen.add("tied")
        if "specials=True" in desc:
            seen.add("specials")
        if list(models[0].buffers()):
            seen.add("buffer")
    want = {"f32", "bf16", "f16", "f64", "mixed", "truncation", "empty model", "transposed", "0 elements", "0-d",
            "two passes", "weights=none", "weights=dirichlet", "weights=signed", "weights=ints",
            "weights=np.float32", "weights=0-d tensors", "weights=special", "specials", "buffer", "tied"}
    assert want <= seen, sorted(want - seen)


def _snapshot(models):
    return [[fz.bits(p).copy() for p in m.parameters()] for m in models]


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["cpu", "cuda"])
@pytest.mark.parametrize("seed", SEEDS)
def test_fedavg_fuzz_case_matches_oracle(seed, where):
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    models, weights, desc = fz.make_case(seed, device="cuda:0" if where == "cuda" else "cpu")
    want = fz.expected(models, weights)
    before = _snapshot(models)
    out = FedAvg.aggregate(models, weights)
    torch.cuda.synchronize()
    got = list(out.parameters())
    ref = list(models[0].parameters())
    assert len(got) == len(want) == len(ref), desc
    for i, (g, r, (d, w)) in enumerate(zip(got, ref, want)):
        ctx = "%s: parameter %d" % (desc, i)
        assert g.dtype == r.dtype and fz.NAME[g.dtype] == d, ctx
        assert g.shape == r.shape and g.stride() == r.stride(), ctx
        assert g.device == r.device and g.requires_grad == r.requires_grad, ctx
        assert g.data_ptr() != r.data_ptr() or g.numel() == 0, ctx
        assert same_bits(fz.bits(g), w, d), ctx
    for b, rb in zip(out.buffers(), models[0].buffers()):
        assert torch.equal(b.cpu(), rb.cpu()) and b.device == rb.device, desc
    after = _snapshot(models)
    for k, (x, y) in enumerate(zip(before, after)):
        assert all(np.array_equal(a, b) for a, b in zip(x, y)), "%s: model %d changed" % (desc, k)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(fz.N_LARGE))
def test_fedavg_large_host_round_fuzz(seed):
    """Rounds above the small-round bound through the chunked host paths (fuzz_cases.make_large_case)."""
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    models, weights, desc = fz.make_large_case(seed)
    want = fz.expected(models, weights)
    out = FedAvg.aggregate(models, weights)
    got = list(out.parameters())
    ref = list(models[0].parameters())
    assert len(got) == len(want), desc
    for i, (g, r, (d, w)) in enumerate(zip(got, ref, want)):
        assert g.device.type == "cpu" and g.shape == r.shape and g.stride() == r.stride(), "%s: parameter %d" % (desc, i)
        assert same_bits(fz.bits(g), w, d), "%s: parameter %d" % (desc, i)


@pytest.mark.gpu
def test_concurrent_device_rounds_from_threads():
    """Four threads, each on a stream of its own, run fuzz rounds of device models back to back with no
    host synchronisation between their rounds: the table ring (8 slots, one event per 4 calls) and the
    upload policy are shared by every thread.  Every round's result against the C oracle afterwards."""
    import threading

    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    seeds = [s for s in SEEDS if len(fz.make_case(s)[0]) >= 33][:6]
    cases = [fz.make_case(s, device="cuda:0") for s in seeds]
    wants = [fz.expected(m, w) for m, w, _ in cases]
    results, errors = [], []

    def worker(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for r in range(12):
                    c = (t + r) % len(cases)
                    models, weights, _ = cases[c]
                    results.append((c, FedAvg.aggregate(models, weights), s))
        except Exception as e:  # noqa: BLE001  (re-raised below)
            errors.append(e)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not errors, errors[0]
    torch.cuda.synchronize()
    assert len(results) == 48
    for c, out, _ in results:
        for i, (g, (d, w)) in enumerate(zip(out.parameters(), wants[c])):
            assert same_bits(fz.bits(g), w, d), "%s: parameter %d" % (cases[c][2], i)
