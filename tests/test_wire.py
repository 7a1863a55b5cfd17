"""Wire format (§8 f1/f3): decoding the reference's serialize_model bytes without
executing the payload, and producing bytes in the same format."""
import collections
import ctypes
import io
import json
import os
import pickle

import numpy as np
import pytest
import torch
from torch import nn

from oracle.fedavg_oracle import fedavg_bits, same_bits

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "wire_spambase_n4.npz")


def _wire_case():
    z = np.load(GOLDEN)
    peers = [z["peer_%d" % k].tobytes() for k in range(4)]
    return peers, z["out"].tobytes(), [float(x) for x in z["weights"]], json.loads(str(z["param_names"]))


def test_decode_reference_payloads_and_pin_the_average():
    from accdfl_amd.core import wire

    peers, out, weights, names = _wire_case()
    sds = [wire.loads_state_dict(b) for b in peers]
    want = wire.loads_state_dict(out)
    assert list(sds[0].keys()) == names == list(want.keys())
    for name in names:
        got = fedavg_bits([sd[name].numpy().reshape(-1) for sd in sds], weights, "f32")
        assert same_bits(got, want[name].numpy().reshape(-1), "f32"), name


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned > /tmp/accdfl_amd_pwned",))


def test_refuses_foreign_globals():
    from accdfl_amd.core import wire

    payload = pickle.dumps({"w": _Evil()})
    if os.path.exists("/tmp/accdfl_amd_pwned"):
        os.remove("/tmp/accdfl_amd_pwned")
    with pytest.raises(wire.UnsafePayloadError):
        wire.loads_state_dict(payload)
    assert not os.path.exists("/tmp/accdfl_amd_pwned")
    with pytest.raises(wire.UnsafePayloadError):
        wire.loads_state_dict(pickle.dumps([1, 2, 3]))  # not a state dict


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
def test_round_trip_every_dtype_with_buffers(dtype):
    from accdfl_amd.core import wire

    m = nn.Sequential(nn.Linear(7, 5), nn.BatchNorm1d(5)).to(dtype)
    b = wire.serialize_model(m)
    sd = wire.loads_state_dict(b)
    ref = m.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k in ref:
        assert sd[k].dtype == ref[k].dtype and torch.equal(sd[k], ref[k]), k
    # the reference's own decoder (pickle.loads + load_state_dict) reads our bytes
    m2 = nn.Sequential(nn.Linear(7, 5), nn.BatchNorm1d(5)).to(dtype)
    m2.load_state_dict(pickle.loads(b))
    assert all(torch.equal(p, q) for p, q in zip(m.parameters(), m2.parameters()))
    assert [n for n, _ in m.named_parameters()] == [n for n, _ in m2.named_parameters()]
    assert [t.data_ptr() for t in wire.parameter_tensors(sd, m)] == [sd[n].data_ptr() for n, _ in m.named_parameters()]


@pytest.mark.gpu
def test_device_model_manager_wire_round():
    """A DFL-style aggregator round on wire bytes: decode -> HBM -> reduce -> bytes,
    against the reference's own FedAvg result for the same payloads."""
    from types import SimpleNamespace

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager

    class LinearModel(nn.Module):  # same parameter names as the reference's spambase model
        def __init__(self):
            super().__init__()
            self.model = nn.Linear(57, 2)

    peers, out, weights, names = _wire_case()
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG),
                            template=LinearModel(), capacity=2)
    for k, b in enumerate(peers):
        mm.process_incoming_serialized(b"peer%d" % k, b)
    mm.process_incoming_serialized(b"peer1", peers[2])  # duplicate peer: ignored
    assert mm.slab.n == 4
    model = mm.aggregate_trained_models(weights)
    want = wire.loads_state_dict(out)
    for name, p in model.named_parameters():
        assert same_bits(p.detach().numpy(), want[name].numpy(), "f32"), name
    back = wire.loads_state_dict(mm.aggregate_serialized(weights))
    for name in names:
        assert same_bits(back[name].numpy(), want[name].numpy(), "f32"), name


@pytest.mark.gpu
@pytest.mark.parametrize("block", [4096, 60_000])
def test_multi_tensor_eva_blocks_into_the_slab(block):
    """Peers of a many-tensor model (a GNLeNet-sized layout) arriving as EVA block lists: every tensor
    that crosses a block is gathered into the peer's ONE page-locked ingress buffer, each at its own
    offset, and must be read from there (round 5's fuzz found every gathered tensor after the first
    viewing the buffer's first bytes).  The round against the C oracle, bit for bit."""
    from types import SimpleNamespace

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager
    from c_oracle import c_wsum

    shapes = [(32, 3, 5, 5), (32,), (32, 32, 5, 5), (32,), (64, 32, 5, 5), (64,), (10, 1024), (10,)]

    class Net(nn.Module):
        def __init__(self, seed):
            super().__init__()
            g = torch.Generator().manual_seed(seed)
            for i, s in enumerate(shapes):
                setattr(self, "p%d" % i, nn.Parameter(torch.randn(s, generator=g)))

    models = [Net(k) for k in range(5)]
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG),
                            template=Net(99), capacity=2)
    for k, m in enumerate(models):
        data = wire.serialize_model(m)
        mm.process_incoming_serialized(b"peer%d" % k, [data[i:i + block] for i in range(0, len(data), block)])
    weights = [0.1, 0.2, 0.3, 0.25, 0.15]
    out = mm.aggregate_trained_models(weights)
    for i, p in enumerate(out.parameters()):
        want = c_wsum([list(m.parameters())[i].detach().reshape(-1).numpy() for m in models], weights, "f32")
        assert same_bits(p.detach().reshape(-1).numpy(), want, "f32"), "parameter %d" % i


def _layout_module(name, dtype, seed):
    """A module with the parameter and buffer layout `name` of tests/golden/layouts.json (the reference's
    models' state-dict layouts), seeded values."""
    lay = json.load(open(os.path.join(os.path.dirname(GOLDEN), "layouts.json")))[name]
    m = nn.Module()
    g = torch.Generator().manual_seed(seed)
    m.ps = nn.ParameterList([nn.Parameter((torch.randn(s, generator=g) * 0.05).to(dtype)) for _, s, _ in lay["params"]])
    for j, (_, s, d) in enumerate(lay["buffers"]):
        m.register_buffer("b%d" % j, torch.randn(s, generator=g).to(getattr(torch, d)) if d != "int64"
                          else torch.full(s, seed + j, dtype=torch.int64))
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["blocks", "bytes", "memoryview"])
def test_real_layout_round_through_the_native_ingress(form):
    """4 google_speech ResNet-34 bf16 peers (110 parameters, 108 BN buffers) through
    the native ingress (one scan, one batched gather, ONE slab copy per peer; the peers' state dicts never
    built), then aggregate_serialized and aggregate_trained_models against FedAvg.aggregate of the same
    modules on the device, bit for bit, with the first arrival's buffers."""
    from types import SimpleNamespace

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg
    from accdfl_amd.core.model_manager import DeviceModelManager

    models = [_layout_module("google_speech_resnet34", torch.bfloat16, 10 + k) for k in range(4)]
    w = [float(x) for x in np.random.default_rng(4).dirichlet(np.ones(4))]
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG),
                            template=_layout_module("google_speech_resnet34", torch.bfloat16, 0), capacity=4)
    want = FedAvg.aggregate([m.cuda() for m in models], w)
    torch.cuda.synchronize()
    models = [m.cpu() for m in models]
    for rnd in range(2):  # the second round reuses the ingress buffers and the slab
        mm.reset_incoming_trained_models()
        for k, m in enumerate(models):
            data = wire.serialize_model(m)
            payload = {"blocks": wire.payload_blocks(data, 60_000), "bytes": data, "memoryview": memoryview(data)}[form]
            mm.process_incoming_serialized(b"peer%d" % k, payload)
        peers = list(mm.incoming_trained_models.values())
        assert mm.slab.n == 4 and all(p._sd is None for p in peers), "the native path builds no state dict"
        direct = wire.loads_state_dict(mm.aggregate_serialized(w))
        out = mm.aggregate_trained_models(w)
        assert all(p._sd is None for p in peers[1:])  # only models[0]'s buffers were read
        for (name, p), q in zip(want.named_parameters(), out.parameters()):
            assert torch.equal(p.detach().cpu().view(torch.int16), q.detach().view(torch.int16)), (rnd, name)
            assert torch.equal(p.detach().cpu().view(torch.int16), direct[name].view(torch.int16)), (rnd, name)
        for name, b in models[0].named_buffers():
            assert torch.equal(direct[name], b) and torch.equal(dict(out.named_buffers())[name], b), (rnd, name)


@pytest.mark.gpu
def test_ingress_falls_back_for_strided_parameters():
    """A payload whose parameter is a transposed view (its storage is not the parameter's dense bytes):
    the native row layout refuses it and the Python decoder stages the round, bit-exact."""
    from types import SimpleNamespace

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager
    from c_oracle import c_wsum

    class Net(nn.Module):
        def __init__(self, seed):
            super().__init__()
            g = torch.Generator().manual_seed(seed)
            self.a = nn.Parameter(torch.randn(70, 300, generator=g).t())  # strides (1, 300)
            self.b = nn.Parameter(torch.randn(5000, generator=g))

    models = [Net(k) for k in range(3)]
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG),
                            template=Net(99), capacity=3)
    for k, m in enumerate(models):
        data = wire.serialize_model(m)
        sc = wire.scan_state_dict(data)
        names, shapes = mm._row_spec()
        assert sc is not None and sc.row_layout(names, torch.float32, shapes) is None
        mm.process_incoming_serialized(b"p%d" % k, wire.payload_blocks(data, 4096))
    assert mm.slab.n == 3 and all(p._sd is not None for p in mm.incoming_trained_models.values())
    w = [0.5, 0.3, 0.2]
    out = mm.aggregate_trained_models(w)
    for i, p in enumerate(out.parameters()):
        want = c_wsum([list(m.parameters())[i].detach().contiguous().reshape(-1).numpy() for m in models], w, "f32")
        assert same_bits(p.detach().contiguous().reshape(-1).numpy(), want, "f32"), i


def test_device_source_entries_encode_like_tensors():
    """wire.DeviceSource (aggregate_serialized's parameter entries): small entries go through the CPU
    like any tensor, so a state dict whose entries are slices of one flat tensor encodes to exactly
    the objects of the plain state dict (CPU: the flat tensor stands in for the averaged row)."""
    from accdfl_amd.core import wire

    flat = torch.randn(3 * 40 + 7, generator=torch.Generator().manual_seed(1))
    sd_plain = collections.OrderedDict([("a", flat[:120].view(3, 40).clone()), ("b", flat[120:].clone()),
                                        ("steps", torch.tensor(5))])
    sd_dev = collections.OrderedDict([("a", wire.DeviceSource(flat, 0, (3, 40))), ("b", wire.DeviceSource(flat, 120, (7,))),
                                      ("steps", torch.tensor(5))])
    for got in (wire.loads_state_dict(wire.dumps_state_dict(sd_dev)), pickle.loads(wire.dumps_state_dict(sd_dev))):
        assert list(got.keys()) == ["a", "b", "steps"]
        for k in sd_plain:
            assert torch.equal(got[k], sd_plain[k]), k


class _ConvBN(nn.Module):
    def __init__(self, seed, dtype):
        super().__init__()
        torch.manual_seed(seed)
        self.conv = nn.Conv2d(64, 128, 3).to(dtype)             # 73 728 weights: a device-sourced entry
        self.bn = nn.BatchNorm2d(128).to(dtype)                  # small params + buffers
        self.fc = nn.Linear(512, 300).to(dtype)                 # 153 600 weights
        with torch.no_grad():
            self.bn.running_mean.fill_(float(seed))
            self.bn.num_batches_tracked.fill_(seed)


class _Tied(nn.Module):
    """A module whose parameter is listed once by parameters() but under two state-dict keys."""

    def __init__(self, seed, dtype):
        super().__init__()
        torch.manual_seed(seed)
        self.enc = nn.Linear(300, 400).to(dtype)
        self.dec = nn.Linear(400, 300, bias=False).to(dtype)
        self.dec.weight = nn.Parameter(self.enc.weight.detach().t().contiguous())
        self.head = nn.Module()
        self.head.weight = self.enc.weight  # alias: state_dict lists it as enc.weight and head.weight


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("peers_as", ["wire", "modules", "device_modules", "tied", "wire_tied"])
def test_aggregate_serialized_straight_from_hbm(dtype, peers_as):
    """VERDICT r02 missing 4: aggregate_serialized copies the averaged parameters from HBM straight
    into the payload (wire.DeviceSource), without the result module; the payload decodes — with the
    reference's own pickle.loads too — to exactly serialize_model(aggregate_trained_models()): the
    same keys in order, the same devices, every parameter bit for bit, the first arrival's buffers.
    ADVICE r03: module peers already in HBM (the payload keeps their tensors' device) and tied
    parameters (every alias key carries the average)."""
    from types import SimpleNamespace

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager

    mk = _Tied if peers_as in ("tied", "wire_tied") else _ConvBN
    models = [mk(k + 1, dtype) for k in range(5)]
    if peers_as == "device_modules":
        models = [m.cuda() for m in models]
    w = [float(x) for x in np.random.default_rng(7).dirichlet(np.ones(5))]
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG),
                            template=mk(0, dtype), capacity=5)
    for k, m in enumerate(models):
        if peers_as in ("wire", "wire_tied"):  # a tied parameter: one tensor under two keys of the payload
            mm.process_incoming_serialized(b"p%d" % k, wire.payload_blocks(wire.serialize_model(m), 60_000))
        else:
            mm.process_incoming_trained_model(b"p%d" % k, m)
    assert mm._uniform()
    direct = mm.aggregate_serialized(w)
    if peers_as == "device_modules":
        want = pickle.loads(wire.serialize_model(mm.aggregate_trained_models(w)))
        got = pickle.loads(direct)
        assert list(got.keys()) == list(want.keys())
        for k in want:
            assert got[k].device == want[k].device, k
            assert torch.equal(got[k].cpu().view(-1).view(torch.uint8), want[k].cpu().view(-1).view(torch.uint8)), k
        return
    want = wire.loads_state_dict(wire.serialize_model(mm.aggregate_trained_models(w)))
    for got in (wire.loads_state_dict(direct), pickle.loads(direct)):
        assert list(got.keys()) == list(want.keys())
        for k in want:
            assert got[k].dtype == want[k].dtype and got[k].shape == want[k].shape, k
            assert torch.equal(got[k].view(-1).view(torch.uint8), want[k].view(-1).view(torch.uint8)), k
    if peers_as in ("tied", "wire_tied"):
        got = wire.loads_state_dict(direct)
        assert torch.equal(got["head.weight"], got["enc.weight"])
        assert not torch.equal(got["enc.weight"], models[0].enc.weight.detach())  # the average, not peer 0's
    else:
        assert torch.equal(wire.loads_state_dict(direct)["bn.running_mean"], models[0].bn.running_mean)


@pytest.mark.gpu
def test_ingress_slot_is_never_reused_within_a_round():
    """a registry entry removed mid-round must not hand its page-locked ingress buffer
    to the next arrival while a live WirePeer still views another slot — slots only advance
    within a round (the old choice, len(registry), reused the buffer of the last live peer)."""
    from types import SimpleNamespace

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager

    template = nn.Linear(300, 200)
    payloads = []
    for k in range(4):
        torch.manual_seed(k)
        payloads.append(wire.serialize_model(nn.Linear(300, 200)))
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG),
                            template=template, capacity=4)
    for k in range(3):
        mm.process_incoming_serialized(b"peer%d" % k, wire.payload_blocks(payloads[k], 1000))
    live = mm.incoming_trained_models[b"peer2"]
    before = {k: v.clone() for k, v in live.state_dict.items()}
    del mm.incoming_trained_models[b"peer1"]  # removed mid-round
    mm.process_incoming_serialized(b"peer3", wire.payload_blocks(payloads[3], 1000))
    torch.cuda.synchronize()
    for k, v in before.items():
        assert torch.equal(live.state_dict[k], v), k
    # the next round starts over at slot 0 (the buffers are reused, not grown without bound)
    mm.reset_incoming_trained_models()
    mm.process_incoming_serialized(b"peer0", wire.payload_blocks(payloads[0], 1000))
    assert mm._ingress_next == 1 and len(mm._ingress) == 4


@pytest.mark.filterwarnings("ignore:TypedStorage is deprecated")
def test_storage_blob_fast_path_and_fallback():
    """The nested storage blobs are parsed in place (no torch.load pass); a blob in any
    other layout (e.g. the zipfile format) goes to torch.load(weights_only=True); a blob
    naming a foreign global is refused."""
    from accdfl_amd.core import wire

    for dt in (torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int64, torch.bool):
        t = (torch.arange(37) % 3).to(dt)
        storage = t.untyped_storage()
        typed = torch.TypedStorage(wrap_storage=storage, dtype=dt, _internal=True)
        blob = typed.__reduce__()[1][0]  # what pickle.dumps(tensor) embeds
        parsed = wire._parse_storage_blob(blob)
        assert parsed.dtype == dt and parsed.size() == 37
        assert torch.equal(torch.tensor([], dtype=dt).set_(parsed._untyped_storage, 0, (37,), (1,)), t)
        zipped = io.BytesIO()
        torch.save(typed, zipped)  # zipfile layout: not the legacy blob
        back = wire._load_storage_blob(zipped.getvalue())
        assert back.dtype == dt
    evil = pickle.dumps(_Evil())
    with pytest.raises(wire.UnsafePayloadError):
        wire._parse_storage_blob(pickle.dumps(0x1950A86A20F9469CFC6C) + pickle.dumps(1001) + pickle.dumps(
            {"little_endian": True}) + evil)


def test_copy_and_view_modes():
    """copy=False: tensors view the decoded blob in place (the ingress path only reads
    them); copy=True (default): private writable tensors."""
    from accdfl_amd.core import wire

    m = nn.Linear(300, 200)
    data = wire.serialize_model(m)
    views = wire.loads_state_dict(data, copy=False)
    own = wire.loads_state_dict(data)
    assert torch.equal(views["weight"], m.weight.detach()) and torch.equal(own["weight"], m.weight.detach())
    own["weight"].add_(1.0)
    assert torch.equal(wire.loads_state_dict(data)["weight"], m.weight.detach())


def test_vm_matches_unpickler_and_reads_in_place():
    """The state_dict pickle VM: same result as the restricted C unpickler, parameter
    bytes viewed in place in the payload (no copy)."""
    from accdfl_amd.core import wire

    m = nn.Sequential(nn.Conv2d(3, 4, 3), nn.BatchNorm2d(4), nn.Linear(5, 6, bias=False))
    data = wire.serialize_model(m)
    a = wire._vm_loads(data)
    b = wire._StateDictUnpickler(io.BytesIO(data)).load()
    assert list(a.keys()) == list(b.keys()) and a._metadata == b._metadata
    for k in a:
        assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape and torch.equal(a[k], b[k])
    base = np.frombuffer(data, dtype=np.uint8).ctypes.data
    assert base <= a["0.weight"].data_ptr() < base + len(data)


def test_vm_rejects_truncated_and_garbage():
    from accdfl_amd.core import wire

    data = wire.serialize_model(nn.Linear(30, 20))
    for cut in (1, 10, len(data) // 2, len(data) - 1):
        with pytest.raises(Exception):
            wire.loads_state_dict(data[:cut])
    rng = np.random.default_rng(0)
    for _ in range(200):  # random payloads: an exception, never a hang or a crash
        junk = bytes(rng.integers(0, 256, size=int(rng.integers(1, 300)), dtype=np.uint8))
        try:
            wire.loads_state_dict(b"\x80\x04" + junk)
        except Exception:
            pass
    # a REDUCE on anything but an allowed global is refused
    with pytest.raises(wire.UnsafePayloadError):
        wire.loads_state_dict(pickle.dumps({"w": _Evil()}, protocol=4))


@pytest.mark.parametrize("block_size", [1, 7, 1000, 60_000, 10 ** 9])
def test_eva_block_list_decodes_like_the_joined_payload(block_size):
    """An EVA transfer's block list (before the reference's b''.join,
    accdfl/util/eva/transfer/incoming.py:35) decodes to the same state dict as the joined
    bytes; tensors whose bytes cross blocks are gathered into the caller's buffer."""
    from accdfl_amd.core import wire

    torch.manual_seed(block_size % 97)
    m = nn.Sequential(nn.Linear(300, 200), nn.BatchNorm1d(200), nn.Linear(200, 3)).to(torch.bfloat16)
    data = wire.serialize_model(m)
    blocks = wire.payload_blocks(data, block_size)
    arena = torch.empty(len(data), dtype=torch.uint8)
    used = [0]

    def alloc(n):
        a = used[0]
        used[0] = a + (n + 255) // 256 * 256
        return arena[a:a + n]

    want = wire.loads_state_dict(data)
    for kw in ({"alloc": alloc}, {}):
        got = wire.loads_state_dict(blocks, copy=False, **kw)
        assert list(got.keys()) == list(want.keys())
        for k in want:
            assert got[k].dtype == want[k].dtype and torch.equal(got[k], want[k]), k
    if block_size < 60_000:  # the 300 x 200 weight crosses blocks: gathered, not joined
        assert used[0] >= 300 * 200 * 2


def test_dfl_split_without_copies():
    """The DFL message = model bytes + pickled population view, split at model_data_len
    (accdfl/dfl/community.py:587-588): on a memoryview and on a block list, no copy."""
    from accdfl_amd.core import wire

    m = nn.Linear(50, 40)
    model_bytes = wire.serialize_model(m)
    view = pickle.dumps({"peers": [1, 2, 3]})
    msg = model_bytes + view
    mv = memoryview(msg)
    sd = wire.loads_state_dict(mv[:len(model_bytes)], copy=False)
    assert torch.equal(sd["weight"], m.weight.detach())
    head, tail = wire.split_blocks(wire.payload_blocks(msg, 333), len(model_bytes))
    assert b"".join(tail) == view and sum(len(h) for h in head) == len(model_bytes)
    sd2 = wire.loads_state_dict(head, copy=True)
    assert torch.equal(sd2["bias"], m.bias.detach())
    with pytest.raises(ValueError):
        wire.split_blocks([b"abc"], 10)


def test_block_table_and_split_edges(monkeypatch):
    """The per-block bookkeeping (native block_table, or the Python fallback without the extension) on
    mixed blocks — bytes, empty bytes, memoryview halves, bytearray — and split_blocks at every kind of
    boundary: 0, inside a block, exactly at a block end, the total; decoding a payload cut into blocks
    with empty blocks in between still matches the joined bytes."""
    from accdfl_amd import _lib
    from accdfl_amd.core import wire

    data = bytes(range(256)) * 40
    mv = memoryview(data[:1000]).cast("B")
    blocks = [data[1000:1500], b"", mv[:300], bytearray(data[2000:2100]), mv[300:], data[5000:6000]]
    want_lens = [500, 0, 300, 100, 700, 1000]
    joined = b"".join(bytes(b) for b in blocks)
    for native in (True, False):
        if not native:
            monkeypatch.setattr(_lib, "walk_module", lambda: None)
        elif _lib.walk_module() is None:
            continue
        addrs, lens = wire._block_table(blocks)
        assert lens.tolist() == want_lens
        for a, ln, b in zip(addrs.tolist(), lens.tolist(), blocks):
            if ln:
                assert ctypes.string_at(a, ln) == bytes(b)
        for n in (0, 1, 499, 500, 800, 900, 1600, len(joined) - 1, len(joined)):
            head, tail = wire.split_blocks(blocks, n)
            assert b"".join(bytes(b) for b in head) == joined[:n], n
            assert b"".join(bytes(b) for b in tail) == joined[n:], n
        with pytest.raises(ValueError):
            wire.split_blocks(blocks, len(joined) + 1)
        m = nn.Linear(64, 33)
        payload = wire.serialize_model(m)
        cut = wire.payload_blocks(payload, 97)
        cut = [x for b in cut for x in (b, b"")]  # empty blocks between every two
        sd = wire.loads_state_dict(cut, copy=True)
        assert torch.equal(sd["weight"], m.weight.detach()) and torch.equal(sd["bias"], m.bias.detach())


def test_block_list_refuses_foreign_globals():
    from accdfl_amd.core import wire

    payload = pickle.dumps({"w": _Evil()})
    with pytest.raises(wire.UnsafePayloadError):
        wire.loads_state_dict(wire.payload_blocks(payload, 5))
    with pytest.raises(wire.UnsafePayloadError):
        wire.loads_state_dict(wire.payload_blocks(wire.serialize_model(nn.Linear(3, 2)), 64)[:-1])  # truncated


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16, torch.float64])
def test_single_copy_serializer_is_the_reference_format(dtype):
    """serialize_model writes tensors of >= 64 KiB with one copy (dumps_state_dict); the bytes
    decode with the reference's own path — plain pickle.loads, i.e. torch's legacy
    _load_from_bytes per storage, then load_state_dict (accdfl/core/models/__init__.py:13-16) —
    to the same tensors, dtypes, shapes and _metadata, and with our restricted decoder."""
    from accdfl_amd.core import wire

    torch.manual_seed(3)
    m = nn.Sequential(nn.Linear(300, 200), nn.BatchNorm1d(200), nn.Linear(200, 3)).to(dtype)
    ref = m.state_dict()
    data = wire.serialize_model(m)
    assert b"_load_from_bytes" in data and b"_rebuild_tensor_v2" in data
    sd = pickle.loads(data)
    assert list(sd.keys()) == list(ref.keys()) and sd._metadata == ref._metadata
    for k in ref:
        assert sd[k].dtype == ref[k].dtype and torch.equal(sd[k], ref[k]), k
    m2 = nn.Sequential(nn.Linear(300, 200), nn.BatchNorm1d(200), nn.Linear(200, 3)).to(dtype)
    m2.load_state_dict(sd)
    for k, v in wire.loads_state_dict(data).items():
        assert torch.equal(v, ref[k]), k
    # a tensor that does not own its storage (a view) takes the stock pickler, same result
    view_sd = {"v": torch.arange(40_000, dtype=torch.float32)[7:30_007]}
    assert torch.equal(pickle.loads(wire.dumps_state_dict(view_sd))["v"], view_sd["v"])
