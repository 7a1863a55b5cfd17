"""Seeded random state dicts through the wire format (accdfl/core/models/__init__.py:9-16:
serialize_model = pickle.dumps(model.state_dict()), unserialize_model = pickle.loads +
load_state_dict), on the CPU:

* the reference's own encoder (pickle.dumps) -> wire.loads_state_dict, from bytes, from a memoryview
  and from EVA-style block lists of random sizes, in copy and view modes;
* wire.dumps_state_dict -> the reference's own decoder (pickle.loads) and -> wire.loads_state_dict.

Entries: float32 / float64 / bfloat16 / float16 / int64 / int32 / int8 / uint8 / bool tensors of 0-3
dimensions, empty ones, transposed and sliced views (strides and storage offsets), two entries
sharing one storage, IEEE specials; every decoded entry must have the dtype, shape, strides and bits
of the original."""
import pickle
from collections import OrderedDict

import numpy as np
import pytest
import torch

from accdfl_amd.core import wire

_DTYPES = [torch.float32, torch.float64, torch.bfloat16, torch.float16, torch.int64, torch.int32, torch.int8,
           torch.uint8, torch.bool]
_BITS = {torch.float32: torch.int32, torch.float64: torch.int64, torch.bfloat16: torch.int16, torch.float16: torch.int16}
N_CASES = 60


def _tensor(rng, dtype):
    numel = int([0, 1, 2, 7, 64, 1000, 4097, 70_001][rng.integers(8)])
    dims = int(rng.integers(0, 4)) if numel == 1 else int(rng.integers(1, 4))
    if dtype.is_floating_point:
        x = torch.from_numpy(rng.standard_normal(numel)).to(dtype)
        if numel and rng.integers(0, 3) == 0:
            x[int(rng.integers(numel))] = float(["nan", "inf", "-inf"][rng.integers(3)])
    elif dtype == torch.bool:
        x = torch.from_numpy(rng.integers(0, 2, size=numel).astype(bool))
    else:
        info = torch.iinfo(dtype)
        x = torch.from_numpy(rng.integers(max(info.min, -1 << 40), min(info.max, 1 << 40), size=numel)).to(dtype)
    if dims == 0:
        return x.reshape(())
    if dims == 1 or numel == 0:
        return x
    a = [d for d in range(1, min(numel, 300) + 1) if numel % d == 0]
    r = int(a[rng.integers(len(a))])
    t = x.view(r, numel // r)
    form = rng.integers(0, 4)
    if form == 0:
        return t.t()                      # transposed: non-contiguous strides
    if form == 1 and t.shape[1] > 2:
        return t[:, 1::2]                 # strided slice with a storage offset
    if form == 2 and dims == 3 and t.shape[1] % 2 == 0:
        return t.view(r, 2, -1)
    if form == 3 and t.shape[0] > 1:
        return t[1:]                      # contiguous, but a storage offset and a larger storage
    return t


def _state_dict(rng):
    sd = OrderedDict()
    for i in range(int(rng.integers(1, 9))):
        sd["t%d" % i] = _tensor(rng, _DTYPES[rng.integers(len(_DTYPES))])
    if rng.integers(0, 3) == 0:  # an entry sharing another entry's storage (tied weights)
        k = "t%d" % int(rng.integers(len(sd)))
        sd["tied"] = sd[k]
        return sd, k
    return sd, None


def _same(a: torch.Tensor, b: torch.Tensor, ctx: str):
    assert a.dtype == b.dtype and a.shape == b.shape, ctx
    assert a.numel() == 0 or a.stride() == b.stride(), ctx
    if a.dtype in _BITS:
        assert torch.equal(a.view(_BITS[a.dtype]), b.view(_BITS[b.dtype])), ctx
    else:
        assert torch.equal(a, b), ctx


def _blocks(rng, data: bytes):
    size = int([1, 3, 100, 4096, 60_000][rng.integers(5)])
    return [data[i:i + size] for i in range(0, len(data), size)]


@pytest.mark.parametrize("seed", range(N_CASES))
def test_wire_fuzz(seed):
    rng = np.random.default_rng(5000 + seed)
    sd, tied = _state_dict(rng)

    def check_tie(got, ctx):  # pickle.loads gives the tied entries one storage (one object)
        if tied is not None and sd[tied].numel():
            assert got["tied"].untyped_storage().data_ptr() == got[tied].untyped_storage().data_ptr(), ctx

    ref_bytes = pickle.dumps(sd)  # the reference's serialize_model
    ref = pickle.loads(ref_bytes)  # the reference's decode: views keep their storage and offset
    for name, payload in (("bytes", ref_bytes), ("memoryview", memoryview(ref_bytes)),
                          ("blocks", _blocks(rng, ref_bytes))):
        for copy in (True, False):
            got = wire.loads_state_dict(payload, copy=copy)
            assert list(got) == list(sd), (seed, name)
            for k in sd:
                ctx = "seed %d %s copy=%s entry %s" % (seed, name, copy, k)
                _same(sd[k], got[k], ctx)
                if copy and ref[k].numel():
                    assert got[k].storage_offset() == ref[k].storage_offset(), ctx
                    assert got[k].untyped_storage().nbytes() == ref[k].untyped_storage().nbytes(), ctx
            check_tie(got, "seed %d %s copy=%s: tied entries" % (seed, name, copy))
    # a block list gathered into ONE bump-allocated buffer (the DeviceModelManager's ingress path):
    # every gathered tensor must view its own part of the buffer
    blocks = _blocks(rng, ref_bytes)
    buf = torch.zeros(len(ref_bytes) + 256 * (len(sd) + 1), dtype=torch.uint8)
    off = [0]

    def alloc(nbytes):
        a = off[0]
        off[0] = a + (nbytes + 255) // 256 * 256
        return buf[a:a + nbytes]

    got = wire.loads_state_dict(blocks, copy=False, alloc=alloc)
    for k in sd:
        _same(sd[k], got[k], "seed %d blocks into one ingress buffer, entry %s" % (seed, k))
    check_tie(got, "seed %d blocks into one ingress buffer: tied entries" % seed)
    ours = wire.dumps_state_dict(sd)
    for name, got in (("pickle.loads", pickle.loads(ours)), ("wire", wire.loads_state_dict(ours))):
        assert list(got) == list(sd), (seed, name)
        for k in sd:
            _same(sd[k], got[k], "seed %d dumps_state_dict -> %s entry %s" % (seed, name, k))
        check_tie(got, "seed %d dumps_state_dict -> %s: tied entries" % (seed, name))


@pytest.mark.parametrize("numel", [1, 5, 1000])
@pytest.mark.parametrize("path", ["template", "general"])
def test_tied_device_source_pickles_once(numel, path):
    """One small DeviceSource (< 64 KiB) listed under two keys (a tied parameter of the averaged model):
    pickle.dumps of the equivalent dict ties the two entries, so the payload must too — through the layout
    template, and through the general path (an entry that is a view forces it; the small DeviceSource is
    then encoded through the CPU, once)."""
    flat = torch.arange(numel + 3, dtype=torch.float32)
    src = wire.DeviceSource(flat, 3, (numel,))
    sd = OrderedDict([("a", src), ("b", src), ("c", torch.ones(2))])
    if path == "general":
        sd["d"] = torch.randn(4, 4)[1:]
    assert (wire._template_plan(sd) is None) == (path == "general")
    got = pickle.loads(wire.dumps_state_dict(sd))
    assert list(got) == list(sd)
    assert torch.equal(got["a"], flat[3:]) and torch.equal(got["b"], flat[3:])
    assert got["a"].untyped_storage().data_ptr() == got["b"].untyped_storage().data_ptr()


def test_payload_template_is_reused_across_rounds():
    """dumps_state_dict's layout template (round 6): the same layout encoded round after round with new
    values decodes — with the reference's own pickle.loads — to exactly that round's state dict (values,
    dtypes, shapes, ties, _metadata); one template per layout; a layout with a view takes the general
    path."""
    from torch import nn

    m = nn.Sequential(nn.Conv2d(3, 4, 3), nn.BatchNorm2d(4), nn.Linear(4, 2)).to(torch.bfloat16)
    wire._TEMPLATES.clear()
    for r in range(3):
        with torch.no_grad():
            for p in m.parameters():
                p.add_(1.0)
            m[1].running_mean.add_(r)
        sd = m.state_dict()
        sd["tied"] = sd["0.weight"]
        got = pickle.loads(wire.dumps_state_dict(sd))
        assert list(got) == list(sd)
        for k in sd:
            _same(sd[k], got[k], "round %d entry %s" % (r, k))
        assert got["tied"] is got["0.weight"]
        assert got._metadata == sd._metadata
    assert len(wire._TEMPLATES) == 1
    view = OrderedDict(a=torch.randn(4, 4)[1:], b=torch.randn(3))
    assert wire._template_plan(view) is None
    got = pickle.loads(wire.dumps_state_dict(view))
    _same(view["a"], got["a"], "view")
