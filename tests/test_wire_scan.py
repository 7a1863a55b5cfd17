"""The native state-dict scan of wire ingress (csrc/walk.cpp scan_state_dict / span_pieces /
build_state_dict, accdfl_amd.core.wire.StateDictScan) against the reference's own decoder:
``pickle.loads`` of ``serialize_model`` bytes (accdfl/core/models/__init__.py:9-16), on the CPU.

* the seeded random state dicts of test_fuzz_wire (every dtype, 0-3 dimensions, empty tensors,
  transposed / sliced views with storage offsets, tied entries), from bytes, memoryviews and EVA-style
  block lists: the built state dict has pickle.loads's keys, dtypes, shapes, strides, storage offsets,
  storage sizes, bits, ties and ``_metadata``;
* the reference-generated payloads of tests/golden/wire_spambase_n4.npz;
* payloads outside a state dict's pickle (foreign globals, not a dict, truncated or trailing bytes,
  garbage) give None — nothing executed — and the Python decoder keeps its own verdict;
* row_layout: the parameters of a real layout (google_speech ResNet-8 of layouts.json) back to back
  from byte 0, and None for views, shared storages, other dtypes or missing keys."""
import collections
import json
import os
import pickle

import numpy as np
import pytest
import torch
from torch import nn

import test_fuzz_wire as fz

pytestmark = pytest.mark.skipif(
    __import__("accdfl_amd._lib", fromlist=["walk_module"]).walk_module() is None,
    reason="the native walk extension is not built")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(sc):
    """Gather every storage into one fresh buffer (256-byte aligned offsets) and build the state dict."""
    offs = np.cumsum([0] + [-(-n // 256) * 256 for *_, n in sc.storages]).astype(np.int64)
    buf = torch.zeros(int(offs[-1]) + 1, dtype=torch.uint8)
    sc.gather(buf, offs[:-1])
    return sc.state_dict(buf, offs[:-1])


def _same_as_pickle(got, ref, ctx):
    assert list(got) == list(ref), ctx
    for k in ref:
        fz._same(ref[k], got[k], "%s entry %s" % (ctx, k))
        assert got[k].requires_grad == ref[k].requires_grad, (ctx, k)
        if ref[k].numel():
            assert got[k].storage_offset() == ref[k].storage_offset(), (ctx, k)
            assert got[k].untyped_storage().nbytes() == ref[k].untyped_storage().nbytes(), (ctx, k)
    # entries pickle.loads ties (one tensor object) are one tensor here too, and no others
    ids_ref = [next(i for i, j in enumerate(ref) if ref[j] is ref[k]) for k in ref]
    ids_got = [next(i for i, j in enumerate(got) if got[j] is got[k]) for k in got]
    assert ids_ref == ids_got, ctx
    assert getattr(got, "_metadata", None) == getattr(ref, "_metadata", None), ctx


@pytest.mark.parametrize("seed", range(fz.N_CASES))
def test_scan_matches_pickle_loads(seed):
    from accdfl_amd.core import wire

    rng = np.random.default_rng(5000 + seed)
    sd, _ = fz._state_dict(rng)
    data = pickle.dumps(sd)
    ref = pickle.loads(data)
    for name, payload in (("bytes", data), ("memoryview", memoryview(data)), ("blocks", fz._blocks(rng, data))):
        sc = wire.scan_state_dict(payload)
        assert sc is not None, (seed, name)
        _same_as_pickle(_build(sc), ref, "seed %d %s" % (seed, name))


def test_scan_of_module_state_dicts_keeps_metadata_and_requires_grad():
    from accdfl_amd.core import wire

    m = nn.Sequential(nn.Conv2d(3, 4, 3), nn.BatchNorm2d(4), nn.Linear(4, 2))
    sd = m.state_dict()
    sd["grad"] = torch.randn(3, requires_grad=True)  # a plain tensor that requires grad
    data = pickle.dumps(sd)
    got = _build(wire.scan_state_dict(wire.payload_blocks(data, 100)))
    _same_as_pickle(got, pickle.loads(data), "state_dict")
    assert got["grad"].requires_grad and not got["1.running_mean"].requires_grad
    # nn.Parameter entries (state_dict(keep_vars=True)) pickle through torch._utils._rebuild_parameter,
    # which no serialize_model payload names: refused by both decoders
    kv = pickle.dumps(m.state_dict(keep_vars=True))
    assert wire.scan_state_dict(kv) is None
    with pytest.raises(wire.UnsafePayloadError):
        wire.loads_state_dict(kv)
    data = wire.serialize_model(m)  # our single-copy encoder's framing
    _same_as_pickle(_build(wire.scan_state_dict(data)), pickle.loads(data), "serialize_model")


def test_scan_of_reference_payloads():
    """tests/golden/wire_spambase_n4.npz holds serialize_model bytes the reference itself produced."""
    from accdfl_amd.core import wire

    z = np.load(os.path.join(ROOT, "tests", "golden", "wire_spambase_n4.npz"))
    for k in range(4):
        data = z["peer_%d" % k].tobytes()
        _same_as_pickle(_build(wire.scan_state_dict(data)), pickle.loads(data), "reference peer %d" % k)
    data = z["out"].tobytes()
    _same_as_pickle(_build(wire.scan_state_dict(wire.payload_blocks(data, 7))), pickle.loads(data), "reference out")


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned > /tmp/accdfl_amd_scan_pwned",))


def test_scan_refuses_what_is_not_a_state_dict():
    from accdfl_amd.core import wire

    if os.path.exists("/tmp/accdfl_amd_scan_pwned"):
        os.remove("/tmp/accdfl_amd_scan_pwned")
    good = wire.serialize_model(nn.Linear(5, 3))
    cases = {
        "foreign global": pickle.dumps({"w": _Evil()}),
        "nested foreign global": pickle.dumps(collections.OrderedDict(w=torch.ones(2), x=_Evil())),
        "list": pickle.dumps([1, 2, 3]),
        "dict of ints": pickle.dumps({"a": 1}),
        "int key": pickle.dumps({1: torch.ones(2)}),
        "trailing bytes": good + b"\x00",
        "garbage": bytes(range(256)) * 4,
        "empty": b"",
    }
    for cut in (1, 2, 10, len(good) // 3, len(good) // 2, len(good) - 1):
        cases["truncated at %d" % cut] = good[:cut]
    for name, payload in cases.items():
        assert wire.scan_state_dict(payload) is None, name
        assert wire.scan_state_dict(wire.payload_blocks(payload, 5)) is None, name
    assert not os.path.exists("/tmp/accdfl_amd_scan_pwned")
    with pytest.raises(wire.UnsafePayloadError):  # the Python decoder keeps its verdict
        wire.loads_state_dict(cases["foreign global"])


def test_scan_refuses_a_storage_blob_with_a_foreign_global():
    """A storage blob whose persistent id names a class other than torch.<X>Storage."""
    from accdfl_amd.core import wire

    good = wire.serialize_model(nn.Linear(5, 3))
    bad = good.replace(b"FloatStorage", b"FloatStorXge")
    assert len(bad) == len(good) and bad != good
    assert wire.scan_state_dict(bad) is None
    with pytest.raises(Exception):
        wire.loads_state_dict(bad)


def test_span_pieces_against_the_joined_payload():
    from accdfl_amd import _lib
    from accdfl_amd.core import wire

    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, size=100_003, dtype=np.uint8).tobytes()
    for size in (1, 7, 4096, 60_000, 200_000):
        blocks = wire.payload_blocks(data, size)
        addrs, lens = wire._block_table(blocks)
        src = np.array([0, 5, 99_999, 12_345, 100_003], dtype=np.int64)
        n = np.array([100_003, 17, 4, 60_001, 0], dtype=np.int64)
        out = torch.zeros(int(n.sum()), dtype=torch.uint8)
        dst = np.concatenate(([0], np.cumsum(n[:-1]))).astype(np.int64) + out.data_ptr()
        d, s, ln = _lib.walk_module().span_pieces(addrs, lens, src, n, dst)
        assert int(ln.sum()) == int(n.sum())
        _lib.host_copy_batch(d, s, ln)
        want = b"".join(data[a:a + k] for a, k in zip(src.tolist(), n.tolist()))
        assert out.numpy().tobytes() == want, size
        with pytest.raises(ValueError):
            _lib.walk_module().span_pieces(addrs, lens, np.array([100_000], np.int64), np.array([4], np.int64),
                                           np.array([out.data_ptr()], np.int64))


def _resnet8_like():
    lay = json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))["cifar10_resnet8"]
    m = nn.Module()
    g = torch.Generator().manual_seed(5)
    m.ps = nn.ParameterList([nn.Parameter(torch.randn(s, generator=g)) for _, s, _ in lay["params"]])
    for j, (_, s, d) in enumerate(lay["buffers"]):
        m.register_buffer("b%d" % j, torch.full(s, float(j), dtype=getattr(torch, d)))
    return m


@pytest.mark.parametrize("native", [True, False])
def test_row_layout_puts_the_parameters_back_to_back(native):
    from accdfl_amd.core import wire

    m = _resnet8_like()
    names = [n for n, _ in m.named_parameters()]
    shapes = [tuple(p.shape) for p in m.parameters()]
    sc = wire.scan_state_dict(wire.payload_blocks(wire.serialize_model(m), 60_000))
    offsets, total, row = sc.row_layout(names, torch.float32, shapes, native=native)
    buf = torch.zeros(total, dtype=torch.uint8)
    sc.gather(buf, offsets)
    want = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert row == want.numel() * 4
    assert torch.equal(buf[:row].view(torch.float32), want)
    got = sc.state_dict(buf, offsets)
    _same_as_pickle(got, pickle.loads(wire.serialize_model(m)), "row layout")
    param_storages = {sc.entries[n][1] for n in names}
    others = [i for i in range(len(sc.storages)) if i not in param_storages]
    assert len(others) == len(list(m.buffers())) and all(offsets[i] % 256 == 0 and offsets[i] >= row for i in others)
    # not a row: another dtype, another shape, a key the payload lacks
    assert sc.row_layout(names, torch.bfloat16, shapes, native=native) is None
    assert sc.row_layout(names, torch.float32, [shapes[0][::-1]] + shapes[1:], native=native) is None
    assert sc.row_layout(names + ["missing"], torch.float32, shapes + [(1,)], native=native) is None


@pytest.mark.parametrize("native", [True, False])
def test_row_layout_refuses_views_and_shared_storages(native):
    from accdfl_amd.core import wire

    base = torch.randn(6, 4)
    sd = collections.OrderedDict(a=base.t(), b=torch.randn(3))  # a strided view
    sc = wire.scan_state_dict(pickle.dumps(sd))
    assert sc.row_layout(["a", "b"], torch.float32, [(4, 6), (3,)], native=native) is None
    sd = collections.OrderedDict(a=base[1:], b=torch.randn(3))  # a storage offset
    sc = wire.scan_state_dict(pickle.dumps(sd))
    assert sc.row_layout(["a", "b"], torch.float32, [(5, 4), (3,)], native=native) is None
    t = torch.randn(3)
    sd = collections.OrderedDict(a=t, b=t)  # one tensor under two parameter names
    sc = wire.scan_state_dict(pickle.dumps(sd))
    assert sc.row_layout(["a", "b"], torch.float32, [(3,), (3,)], native=native) is None
    assert sc.row_layout(["a"], torch.float32, [(3,)], native=native) is not None


@pytest.mark.parametrize("seed", range(4 * int(os.environ.get("ACCDFL_AMD_FUZZ_SCALE", "1"))))
def test_scan_of_mutated_payloads_agrees_with_the_python_decoder(seed):
    """Untrusted bytes: seeded mutations of state-dict payloads (byte flips, deletions, insertions, small
    field changes; as bytes and as block lists) never crash the native scan, and whatever it accepts the
    Python decoder accepts too and decodes to the same state dict (dtypes, shapes, strides, storage
    offsets and sizes, bits, ties, _metadata).  Everything else it leaves to the Python decoder."""
    import warnings

    from accdfl_amd.core import wire

    rng = np.random.default_rng(900 + seed)
    accepted = 0
    for it in range(80):
        sd, _ = fz._state_dict(np.random.default_rng(int(rng.integers(1 << 30))))
        data = bytearray(pickle.dumps(sd) if rng.integers(2) else wire.dumps_state_dict(sd))
        kind = int(rng.integers(4))
        for _ in range(int(rng.integers(1, 4))):
            if kind == 0 and data:
                data[int(rng.integers(len(data)))] = int(rng.integers(256))
            elif kind == 1 and data:
                i = int(rng.integers(len(data)))
                del data[i:i + int(rng.integers(1, 64))]
            elif kind == 2:
                i = int(rng.integers(len(data) + 1))
                data[i:i] = bytes(rng.integers(0, 256, int(rng.integers(1, 16)), dtype=np.uint8))
            elif data:
                i = int(rng.integers(len(data)))
                data[i] = (data[i] + int(rng.integers(1, 4))) & 255
        data = bytes(data)
        payload = wire.payload_blocks(data, int(rng.choice([7, 100, 4096, 60_000]))) if rng.integers(2) else data
        sc = wire.scan_state_dict(payload)
        if sc is None:
            continue
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            ref = wire.loads_state_dict(data)  # must not raise: the native scan accepted the payload
        _same_as_pickle(_build(sc), ref, "seed %d mutant %d" % (seed, it))
        accepted += 1
    assert accepted > 5  # the mutants include accepted ones (value bytes changed)


@pytest.mark.parametrize("seed", range(fz.N_CASES))
def test_native_row_layout_matches_the_python_rules(seed):
    """walk.cpp row_layout against StateDictScan's Python rules on the fuzz state dicts: random subsets of
    the keys in random order as the parameter names, their true shapes or perturbed ones, the true dtype
    or another — the same offsets, total and row, or None from both."""
    from accdfl_amd.core import wire

    rng = np.random.default_rng(7000 + seed)
    sd, _ = fz._state_dict(rng)
    sc = wire.scan_state_dict(pickle.dumps(sd))
    keys = list(sd)
    for _ in range(6):
        names = [keys[i] for i in rng.permutation(len(keys))[:int(rng.integers(1, len(keys) + 1))]]
        shapes = [tuple(sd[k].shape) for k in names]
        if rng.integers(3) == 0:
            j = int(rng.integers(len(shapes)))
            shapes[j] = shapes[j] + (1,)
        dtype = sd[names[0]].dtype if rng.integers(4) else torch.float64
        a = sc.row_layout(names, dtype, shapes, native=True)
        b = sc.row_layout(names, dtype, shapes, native=False)
        assert (a is None) == (b is None), (seed, names)
        if a is not None:
            assert np.array_equal(a[0], b[0]) and a[1:] == b[1:], (seed, names)


def test_gather_and_build_refuse_out_of_bounds():
    """The native build checks every view against its storage whoever made the descriptions, and the
    gather refuses offsets outside the destination buffer."""
    from accdfl_amd import _lib
    from accdfl_amd.core import wire

    sd = collections.OrderedDict(a=torch.arange(10, dtype=torch.float32), b=torch.ones(3, dtype=torch.int64))
    sc = wire.scan_state_dict(pickle.dumps(sd))
    buf = torch.zeros(1024, dtype=torch.uint8)
    with pytest.raises(ValueError):
        sc.gather(buf, np.array([0, 1010], dtype=np.int64))
    with pytest.raises(ValueError):
        sc.gather(buf, np.array([-8, 256], dtype=np.int64))
    offs = np.array([0, 256], dtype=np.int64)
    sc.gather(buf, offs)
    assert torch.equal(sc.state_dict(buf, offs)["a"], sd["a"])
    tag, sidx, off, size, stride, rg = sc.entries["a"]
    forged = collections.OrderedDict(a=(tag, sidx, off, (11,), stride, rg))  # one element past the storage
    with pytest.raises(ValueError):
        _lib.walk_module().build_state_dict(buf, offs, forged, sc.storages, collections.OrderedDict)
    forged = collections.OrderedDict(a=(tag, sidx, 1, size, stride, rg))  # shifted by one
    with pytest.raises(ValueError):
        _lib.walk_module().build_state_dict(buf, offs, forged, sc.storages, collections.OrderedDict)
    with pytest.raises(ValueError):
        _lib.walk_module().build_state_dict(buf, np.array([0, 1020], dtype=np.int64), sc.entries, sc.storages,
                                            collections.OrderedDict)


def test_corrupt_lengths_are_refused_without_allocating_them():
    """A few corrupt length bytes must not make either decoder allocate what they claim: a protocol-5
    BYTEARRAY8 claiming 1 TiB, and a legacy storage blob whose element count claims 2^40 elements (torch's
    legacy loader would allocate them) — both refused (UnsafePayloadError) by the Python decoder, None from
    the native scan, in well under a second and without growing the process."""
    import resource
    import time

    from accdfl_amd.core import wire

    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    huge = b"\x80\x05\x96" + (1 << 40).to_bytes(8, "little") + b"abc."
    t = torch.arange(12345, dtype=torch.float32)
    good = pickle.dumps(collections.OrderedDict(w=t))
    field = t.numel().to_bytes(8, "little")
    at = good.index(field, good.index(b"FloatStorage"))
    bad = good[:at] + (1 << 40).to_bytes(8, "little") + good[at + 8:]
    for payload in (huge, bad):
        t0 = time.perf_counter()
        assert wire.scan_state_dict(payload) is None
        with pytest.raises(wire.UnsafePayloadError):
            wire.loads_state_dict(payload)
        assert time.perf_counter() - t0 < 5.0
    assert resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - rss0 < 512 * 1024  # KiB: < 512 MiB more
