"""CPU-side checks: the C-ABI library loads and exports every entry point that
include/dlagg.h declares; host logic mirrors the reference's error behaviour; the
product path refuses to run without a HIP device (no CPU fallback)."""
import ctypes
import os
import re
import time
from collections import OrderedDict

import pytest
import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    text = open(os.path.join(ROOT, "include", "dlagg.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|void|const char\*)\s+(dla_\w+)\s*\(", text, re.M)))


@pytest.fixture(scope="module")
def lib_path():
    from accdfl_amd import _lib

    return _lib.build()


def test_header_declares_entry_points():
    syms = _declared_symbols()
    assert {"dla_wsum", "dla_wsum_ex", "dla_wsum_slab", "dla_wsum_multi", "dla_version",
            "dla_last_error"} <= set(syms)


def test_library_exports_every_declared_symbol(lib_path):
    so = ctypes.CDLL(lib_path)
    for s in _declared_symbols():
        assert hasattr(so, s), s
    from accdfl_amd import _lib

    assert set(_lib.EXPORTED) == set(_declared_symbols())


def test_stale_library_is_refused(lib_path, tmp_path):
    """A library whose embedded build id is not the tree's (built from other sources) fails
    loudly at load instead of running old code."""
    from accdfl_amd import _lib

    data = bytearray(open(lib_path, "rb").read())
    i = data.find(b"dlagg-build-id:") + len(b"dlagg-build-id:")
    data[i] = ord("0") if data[i] != ord("0") else ord("1")
    stale = tmp_path / "libdlagg_stale.so"
    stale.write_bytes(bytes(data))
    assert _lib.file_build_id(str(stale)) != _lib.source_build_id()
    with pytest.raises(RuntimeError, match="stale libdlagg.so"):
        _lib._Lib(str(stale))


def test_library_version_and_argument_errors(lib_path):
    """Calls that fail validation never touch the GPU, so they run here."""
    from accdfl_amd import _lib

    L = _lib.lib()
    assert L.so.dla_version() == 13
    assert L.build_id == _lib.source_build_id() == _lib.file_build_id(lib_path)
    assert L.max_peers_per_pass == 128
    # kernel selection by shape (host-only query): north star, configs[3] share, configs[4] share,
    # configs[2], GNLeNet 8 peers, fp64 north-star shape, few peers, invalid arguments
    assert _lib.select_kernel(0, 8, 25_000_000) == "wsum_vec_kernel"  # capped row-major (r03ag)
    assert _lib.select_kernel(0, 16, 24_500_000) == "wsum_bigtile_kernel"
    assert _lib.select_kernel(0, 64, 21_339) == "wsum_vec_kernel"
    assert _lib.select_kernel(1, 128, 2_662_045) == "wsum_vec_kernel"
    assert _lib.select_kernel(0, 32, 1_690_046) == "wsum_vec_kernel"
    assert _lib.select_kernel(3, 64, 21_339) == "wsum_wide_kernel"
    assert _lib.select_kernel(0, 8, 85_354) == "wsum_stream_kernel"
    assert _lib.select_kernel(3, 8, 12_500_000) == "wsum_bigtile_kernel"
    assert _lib.select_kernel(0, 4, 25_000_000) == "wsum_stream_kernel"
    # big tiles when the input exceeds the 256 MiB Infinity Cache and they fill their last
    # round of 1024 resident waves (>= 80 %), or there is at least one full round (balanced
    # launch: the partial last round goes to segment workgroups)
    assert _lib.select_kernel(0, 16, 12_500_000) == "wsum_bigtile_kernel"
    assert _lib.select_kernel(0, 16, 21_296_355) == "wsum_bigtile_kernel"
    assert _lib.select_kernel(0, 8, 21_300_000) == "wsum_vec_kernel"  # 8 fp32 peers: capped row-major
    assert _lib.select_kernel(3, 8, 21_300_000) == "wsum_bigtile_kernel"  # fp64 keeps the big tile
    assert _lib.select_kernel(0, 8, 3_400_000) == "wsum_stream_kernel"
    assert _lib.select_kernel(0, 32, 3_000_000) == "wsum_vec_kernel"  # 0.72 of one round
    assert _lib.select_kernel(0, 32, 4_110_000) == "wsum_bigtile_kernel"
    assert _lib.select_kernel(0, 32, 8_200_000) == "wsum_bigtile_kernel"
    assert _lib.select_kernel(0, 24, 8_200_000) == "wsum_vec_kernel"
    assert _lib.select_kernel(1, 8, 50_000_000) == "wsum_vec_kernel"  # bf16 / f16: any peer count
    assert _lib.select_kernel(2, 3, 1000) == "wsum_vec_kernel" and _lib.select_kernel(3, 3, 1000) != "wsum_vec_kernel"
    assert _lib.select_kernel(9, 8, 100) == "" and _lib.select_kernel(0, 0, 100) == ""
    # tile of the tile-interleaved PeerSlab (dla_slab_tile_elems, host-only)
    assert _lib.slab_tile_elems(0, 8, 25_000_000) * 4 == 32768
    assert _lib.slab_tile_elems(0, 16, 25_000_000) * 4 == 16384
    assert _lib.slab_tile_elems(1, 128, 2_662_045) * 2 == 4096
    assert _lib.slab_tile_elems(0, 128, 85_354) * 4 == 1024 and _lib.slab_tile_elems(0, 8, 1000) * 4 == 1024
    assert _lib.slab_tile_elems(9, 8, 100) == 0
    # n_peers = 0 -> DLA_E_INVALID with a message
    rc = L.so.dla_wsum(0, None, None, 0, 10, None, None)
    assert rc == -1 and b"n_peers" in L.so.dla_last_error()
    # unknown dtype
    rc = L.so.dla_wsum(9, None, None, 1, 10, None, None)
    assert rc == -1 and b"dtype" in L.so.dla_last_error()
    with pytest.raises(_lib.DlaggError):
        _lib.wsum_ptrs(0, [0], [1.0], 10, 0, 0)  # null peer pointer
    # empty buffers are a no-op (nothing launched)
    _lib.wsum_ptrs(0, [16], [1.0], 0, 16, 0)
    # alias of a non-first peer in a multi-pass (>128 peers) reduce is refused
    ptrs = [4096 * (k + 1) for k in range(130)]
    with pytest.raises(_lib.DlaggError, match="alias"):
        _lib.wsum_ptrs(0, ptrs, [1.0] * 130, 64, ptrs[5], 0)
    # dla_wsum_multi_table: the table size, and argument errors caught before any GPU work
    assert _lib.wsum_multi_table_bytes(110, 128) == (1088 + 110 * 40) + 110 * 128 * 8  # index, records, pointers
    assert _lib.wsum_multi_table_bytes(300, 2) == (1088 + 256 * 40) + (1088 + 44 * 40 + 0) + 300 * 2 * 8
    assert _lib.wsum_multi_table_bytes(3, 0) == 0
    rc = L.so.dla_wsum_multi_table(0, 1, None, None, None, None, 1, None, None, None)
    assert rc == -1 and b"tensor table" in L.so.dla_last_error()
    with pytest.raises(_lib.DlaggError, match="aliases peer 5"):
        _lib.wsum_multi_table_ptrs(0, ptrs, [ptrs[5]], [64], [1.0] * 130, 0, 0, 0)
    # dla_slab_stage: argument errors caught before any copy (row outside the slab, null base / src)
    rc = L.so.dla_slab_stage(0, 4096, 1024, 8, 4, 8, 0, 8192, 100, None)
    assert rc == -1 and b"row" in L.so.dla_last_error()
    rc = L.so.dla_slab_stage(0, None, 1024, 8, 4, 0, 0, 8192, 100, None)
    assert rc == -1
    rc = L.so.dla_slab_stage(0, 4096, 1024, 8, 4, 0, 0, None, 100, None)
    assert rc == -1 and b"src" in L.so.dla_last_error()
    assert L.so.dla_slab_stage(0, 4096, 1024, 8, 4, 0, 0, None, 0, None) == 0  # nothing to copy
    # a range past the slab's 4 tiles of 1024 elements is refused before any copy
    rc = L.so.dla_slab_stage(0, 4096, 1024, 8, 4, 0, 4000, 8192, 97, None)
    assert rc == -1 and b"do not fit" in L.so.dla_last_error()
    rc = L.so.dla_slab_stage(0, 4096, 1024, 8, 4, 0, 4097, 8192, 0, None)
    assert rc == -1 and b"do not fit" in L.so.dla_last_error()
    # launch knobs outside the built set are refused before any launch
    for bad in (_lib.LaunchCfg(3, 0, 0, 0), _lib.LaunchCfg(4, 3, 0, 0), _lib.LaunchCfg(4, 1, 0, 128),
                _lib.LaunchCfg(10, 0, 0, 0), _lib.LaunchCfg(11, 0, 0, 0)):  # 16-byte vec forms: not built
        with pytest.raises(_lib.DlaggError):
            _lib.wsum_ptrs(0, [4096], [1.0], 64, 8192, 0, bad)


def test_host_copy_batch_runs_on_cpu(lib_path):
    """dla_host_copy_batch is host-only: it gathers and scatters here without a GPU."""
    import numpy as np

    from accdfl_amd import _lib

    rng = np.random.default_rng(0)
    srcs = [rng.standard_normal(s).astype(np.float32) for s in (3, 0, 1000, 17)]
    row = np.zeros(sum(a.size for a in srcs), dtype=np.float32)
    dsts, off = [], 0
    for a in srcs:
        dsts.append(row.ctypes.data + off * 4)
        off += a.size
    _lib.host_copy_batch(dsts, [a.ctypes.data for a in srcs], [a.nbytes for a in srcs])
    assert np.array_equal(row, np.concatenate(srcs))
    back = [np.empty_like(a) for a in srcs]
    _lib.host_copy_batch([b.ctypes.data for b in back], dsts, [a.nbytes for a in srcs])
    assert all(np.array_equal(a, b) for a, b in zip(srcs, back))
    with pytest.raises(_lib.DlaggError, match="null"):
        _lib.host_copy_batch([0], [srcs[0].ctypes.data], [12])
    with pytest.raises(_lib.DlaggError, match="negative"):
        _lib.host_copy_batch([row.ctypes.data], [srcs[0].ctypes.data], [-1])


def test_host_round_argument_errors(lib_path):
    """dla_host_round_start / _finish refuse bad tables, pitches and pageable rows before any
    GPU work (the kernel would read them across PCIe)."""
    import numpy as np

    from accdfl_amd import _lib

    rows = np.zeros((2, 64), dtype=np.float32)
    res = np.zeros(64, dtype=np.float32)
    a = np.ones(10, dtype=np.float32)
    ptrs = [a.ctypes.data, a.ctypes.data]
    with pytest.raises(_lib.DlaggError, match="pitch"):
        _lib.host_round_start(0, 2, ptrs, [10], [0.5, 0.5], rows.ctypes.data, 8, res.ctypes.data, 0)
    with pytest.raises(_lib.DlaggError, match="page-locked"):
        _lib.host_round_start(0, 2, ptrs, [10], [0.5, 0.5], rows.ctypes.data, 64, res.ctypes.data, 0)
    with pytest.raises(_lib.DlaggError, match="dtype"):
        _lib.host_round_start(9, 2, ptrs, [10], [0.5, 0.5], rows.ctypes.data, 64, res.ctypes.data, 0)
    with pytest.raises(_lib.DlaggError, match="aligned"):
        _lib.host_round_start(0, 2, ptrs, [10], [0.5, 0.5], rows.ctypes.data + 4, 64, res.ctypes.data, 0)
    with pytest.raises(_lib.DlaggError, match="bad tensor"):
        _lib.host_round_finish(0, [10], res.ctypes.data, [0], 0)


def test_host_reduce_argument_errors(lib_path):
    """dla_host_reduce refuses bad chunk sizes, tables, dtypes and pageable staging before any copy."""
    import numpy as np

    from accdfl_amd import _lib

    st = np.zeros(4 * 64, dtype=np.float32)
    a = np.ones(10, dtype=np.float32)
    out = np.zeros(10, dtype=np.float32)
    ptrs = [a.ctypes.data, a.ctypes.data]
    buf = st.ctypes.data

    def call(dtype=0, chunk=64, tensors=ptrs, outs=(out.ctypes.data,), h_stage=buf, begin=0, end=10):
        _lib.host_reduce(dtype, 2, tensors, [10], [0.5, 0.5], list(outs), begin, end, chunk, h_stage, buf, buf, buf,
                         0, 0)

    with pytest.raises(_lib.DlaggError, match="256 bytes"):
        call(chunk=10)
    with pytest.raises(_lib.DlaggError, match="dtype"):
        call(dtype=9)
    with pytest.raises(_lib.DlaggError, match="null tensor"):
        call(tensors=[a.ctypes.data, 0])
    with pytest.raises(_lib.DlaggError, match="null output"):
        call(outs=(0,))
    with pytest.raises(_lib.DlaggError, match="begin"):
        call(begin=4, end=11)
    with pytest.raises(_lib.DlaggError, match="begin"):
        call(begin=5, end=4)
    with pytest.raises(_lib.DlaggError, match="page-locked"):
        call()
    # the deferred form: outputs are checked only once published, and a flag is required
    L = _lib.lib()
    rc = L.so.dla_host_reduce_deferred(0, 2, 1, (ctypes.c_void_p * 2)(*ptrs), (ctypes.c_int64 * 1)(10),
                                       (ctypes.c_double * 2)(0.5, 0.5), (ctypes.c_void_p * 1)(0), None, 0, 10, 64,
                                       buf, buf, buf, buf, 0, 0)
    assert rc != 0 and b"outs_ready" in L.so.dla_last_error()
    job = ctypes.c_void_p()
    args = (0, 2, 1, (ctypes.c_void_p * 2)(*ptrs), (ctypes.c_int64 * 1)(10), (ctypes.c_double * 2)(0.5, 0.5),
            (ctypes.c_void_p * 1)(0), ctypes.byref(ctypes.c_int(0)), 0, 10, 64, buf, buf, buf, buf, 0, 0)
    assert L.so.dla_host_reduce_launch(0, *args, None) != 0 and b"job is required" in L.so.dla_last_error()
    assert L.so.dla_host_reduce_launch(4096, *args, ctypes.byref(job)) != 0 and job.value is None
    assert b"no HIP device 4096" in L.so.dla_last_error()
    assert L.so.dla_host_reduce_join(None) != 0 and b"null job" in L.so.dla_last_error()
    with pytest.raises(_lib.DlaggError, match="page-locked"):  # not "null output": outs unpublished yet
        _lib.host_reduce(0, 2, ptrs, [10], [0.5, 0.5], (ctypes.c_void_p * 1)(0), 0, 10, 64, buf, buf, buf, buf, 0,
                         0, outs_ready=ctypes.c_int(0))


def test_host_round_tables_must_match_their_counts(lib_path):
    """The bindings refuse pointer / weight tables whose length differs from what the library reads
    (n_peers x n_tensors peers, n_tensors outputs, n_peers weights) before calling it: a short table
    would be read past its end (the round-5 fuzz found a caller passing one output for several tensors)."""
    import numpy as np

    from accdfl_amd import _lib

    a = np.ones(10, dtype=np.float32)
    buf = np.zeros(256, dtype=np.float32).ctypes.data
    two = [a.ctypes.data, a.ctypes.data]
    with pytest.raises(ValueError, match="output pointers for 2 tensors"):
        _lib.host_reduce(0, 2, two * 2, [5, 5], [0.5, 0.5], [a.ctypes.data], 0, 10, 64, buf, buf, buf, buf, 0, 0)
    with pytest.raises(ValueError, match="3 peer pointers for 1 tensors of 2 peers"):
        _lib.host_reduce(0, 2, two + two[:1], [10], [0.5, 0.5], [a.ctypes.data], 0, 10, 64, buf, buf, buf, buf, 0, 0)
    with pytest.raises(ValueError, match="1 weights for 2 peers"):
        _lib.host_reduce(0, 2, two, [10], [0.5], [a.ctypes.data], 0, 10, 64, buf, buf, buf, buf, 0, 0)
    with pytest.raises(ValueError, match="1 weights for 2 peers"):
        _lib.host_round_start(0, 2, two, [10], [0.5], buf, 64, buf, 0)
    with pytest.raises(ValueError, match="2 output pointers for 1 tensors"):
        _lib.host_round_finish(0, [10], buf, [buf, buf], 0)


class _OddModule(nn.Module):
    """Tied weights, nested containers, an LSTM (its own __setstate__ / __getstate__), buffers
    (one non-persistent), a forward hook, plain attributes sharing a dict."""

    def __init__(self):
        super().__init__()
        self.enc = nn.Linear(4, 3)
        self.tied = self.enc
        self.seq = nn.Sequential(nn.Conv2d(3, 4, 3), nn.BatchNorm2d(4), nn.ReLU(), nn.GroupNorm(2, 4))
        self.rnn = nn.LSTM(4, 5)
        self.pl = nn.ParameterList([nn.Parameter(torch.randn(3)), nn.Parameter(torch.randn(2), requires_grad=False)])
        self.cfg = {"a": [1, 2], "b": (3, 4)}
        self.lst = [self.cfg, torch.ones(2)]
        self.name = "x"
        self.register_buffer("steps", torch.tensor(5))
        self.register_buffer("np", torch.zeros(2), persistent=False)
        self.fh = self.register_forward_hook(lambda m, i, o: None)
        # containers the native clone (walk.cpp clone_value) copies itself: a tuple holding a mutable
        # item (a new tuple), a list holding itself, an OrderedDict out of insertion order, a tuple
        # key, a shared tuple of numbers, an empty set
        self.mixed = (1, [2, 3], "s")
        self.loop = [4]
        self.loop.append(self.loop)
        self.od = OrderedDict([("x", 1), ("y", [5]), ("z", 3)])
        self.od.move_to_end("x")
        self.tk = {(1, 2): "a", "b": self.mixed}
        self.nums = (7, 8)
        self.nums2 = self.nums
        self.empty = set()


def _same_structure(x, y, seen):
    if id(x) in seen:
        return
    seen.add(id(x))
    assert type(x) is type(y)
    if isinstance(x, torch.Tensor):
        assert x.shape == y.shape and x.dtype == y.dtype and x.requires_grad == y.requires_grad
        assert x is not y
        if not isinstance(x, nn.Parameter):
            assert torch.equal(x, y)
    elif isinstance(x, nn.Module):
        assert list(x.__dict__) == list(y.__dict__) and x is not y
        for k in x.__dict__:
            _same_structure(x.__dict__[k], y.__dict__[k], seen)
    elif isinstance(x, dict):
        assert list(x) == list(y)
        for k in x:
            _same_structure(x[k], y[k], seen)
    elif isinstance(x, (list, tuple)):
        assert len(x) == len(y)
        for u, v in zip(x, y):
            _same_structure(u, v, seen)
    elif isinstance(x, (set, int, float, str, bool, type(None))):
        assert x == y


@pytest.mark.parametrize("native", [True, False], ids=["native_clone", "python_clone"])
def test_center_copy_is_a_deepcopy(native, monkeypatch):
    """The result module (fedavg.py:20 copy.deepcopy(models[0])) built by _center_copy's module
    clone matches copy.deepcopy attribute for attribute: same types and key order, fresh
    objects, buffers equal, identity preserved (tied weights, a dict shared by two attributes),
    parameters fresh with the same requires_grad, and the copy runs — with the tree's dicts,
    tuples and lists cloned by the walk extension (walk.cpp clone_value) and in Python."""
    import copy

    from accdfl_amd import _lib
    from accdfl_amd.core.gradient_aggregation import fedavg as fa
    from accdfl_amd.core.gradient_aggregation.fedavg import _center_copy

    if native and _lib.walk_module() is None:
        pytest.skip("walk extension not built")
    monkeypatch.setattr(fa, "_NATIVE_CLONE", native)
    m = _OddModule()
    want = copy.deepcopy(m)
    got = _center_copy(m, large=False)
    _same_structure(want, got, set())
    assert got.tied is got.enc and got.lst[0] is got.cfg and got.cfg is not m.cfg
    assert got.mixed is not m.mixed and got.mixed[1] is not m.mixed[1] and got.mixed == m.mixed
    assert got.tk["b"] is got.mixed and list(got.tk) == [(1, 2), "b"]
    assert got.loop is not m.loop and got.loop[1] is got.loop and got.loop[0] == 4
    assert type(got.od) is OrderedDict and list(got.od) == ["y", "z", "x"] and got.od["y"] is not m.od["y"]
    assert got.nums is m.nums and got.nums2 is got.nums  # deepcopy keeps tuples of numbers
    assert got.empty == set() and got.empty is not m.empty
    assert len(got._forward_hooks) == 1 and got._forward_hooks is not m._forward_hooks
    assert [p.requires_grad for p in got.parameters()] == [p.requires_grad for p in m.parameters()]
    assert all(p is not q for p, q in zip(got.parameters(), m.parameters()))
    got.seq(torch.zeros(1, 3, 5, 5))
    got.rnn(torch.zeros(2, 1, 4))
    # the same with the module classes classified first, as every aggregate does (the walk extension then
    # lists the buffers and _center_copy copies them by one gather per dtype): buffers equal, in their own
    # storage, a buffer sharing another's storage left to deepcopy (sharing kept)
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    m = _OddModule()
    m.register_buffer("mean_view", m.seq[1].running_mean[1:3])  # shares the BN buffer's storage
    for cls in {type(x) for x in m.modules()}:
        fa._plain_walk(cls)
    want = copy.deepcopy(m)
    got = _center_copy(m, large=False)
    _same_structure(want, got, set())
    for (name, b), c in zip(m.named_buffers(), got.buffers()):
        assert torch.equal(b, c) and b.untyped_storage().data_ptr() != c.untyped_storage().data_ptr(), name
    assert got.mean_view.untyped_storage().data_ptr() == got.seq[1].running_mean.untyped_storage().data_ptr()
    got.seq[1].running_var.add_(1.0)
    assert not torch.equal(got.seq[1].running_var, m.seq[1].running_var)
    # a parametrized module (its generated class has its own __deepcopy__: the stock path, same memo)
    from torch.nn.utils import parametrizations

    pm = nn.Sequential(parametrizations.weight_norm(nn.Linear(4, 3)), nn.Linear(3, 2))
    want, got = copy.deepcopy(pm), _center_copy(pm, large=False)
    assert type(got[0]) is type(want[0]) and got[0] is not pm[0]
    assert [n for n, _ in got.named_parameters()] == [n for n, _ in pm.named_parameters()]
    assert all(p is not q for p, q in zip(got.parameters(), pm.parameters()))
    assert got(torch.zeros(1, 4)).shape == (1, 2)


def _tiny_models(n):
    return [nn.Linear(4, 2) for _ in range(n)]


def test_fedavg_reference_error_behaviour():
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    with pytest.raises(IndexError):          # fedavg.py:20 models[0] on an empty list
        FedAvg.aggregate([], None)
    with pytest.raises(AssertionError):      # fedavg.py:17
        FedAvg.aggregate(_tiny_models(3), [0.5, 0.5])


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU refusal")
def test_no_cpu_fallback():
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    with pytest.raises(RuntimeError, match="no HIP device"):
        FedAvg.aggregate(_tiny_models(2), None)


def test_plugin_surface_matches_reference():
    from accdfl_amd.core.gradient_aggregation import GradientAggregation, GradientAggregationMethod
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    assert int(GradientAggregationMethod.FEDAVG) == 1
    assert issubclass(FedAvg, GradientAggregation)
    assert isinstance(FedAvg.__dict__["aggregate"], staticmethod)


def test_model_manager_registry_semantics():
    """model_manager.py:42-58: first arrival wins; order = arrival order; selector."""
    from types import SimpleNamespace

    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg
    from accdfl_amd.core.model_manager import ModelManager

    mm = ModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0)
    a, b, c = _tiny_models(3)
    mm.process_incoming_trained_model(b"p2", b)
    mm.process_incoming_trained_model(b"p1", a)
    mm.process_incoming_trained_model(b"p2", c)  # duplicate peer: ignored
    assert list(mm.incoming_trained_models.values()) == [b, a]
    assert mm.get_aggregation_method() is FedAvg
    mm.reset_incoming_trained_models()
    assert mm.incoming_trained_models == {}
    mm2 = ModelManager(None, SimpleNamespace(gradient_aggregation=99), 0)
    assert mm2.get_aggregation_method() is None


def test_bucket_bounds():
    from accdfl_amd.core.sharding import bucket_bounds

    for n in (0, 1, 63, 64, 65, 1000, 25_000_000, 21_296_355):
        for world in (1, 2, 3, 4, 8):
            b = bucket_bounds(n, world, 64)
            assert len(b) == world
            assert b[0][0] == 0 and b[-1][1] == n
            for (s0, e0), (s1, e1) in zip(b, b[1:]):
                assert e0 == s1
            for s, e in b:
                assert s % 64 == 0 or s == n
                assert s <= e


def test_shard_range_matches_bucket_bounds(lib_path):
    """dla_shard_range (host-only) splits exactly like core/sharding.bucket_bounds: contiguous
    buckets whose starts are multiples of 256 bytes, covering every element once."""
    from accdfl_amd import _lib
    from accdfl_amd.core.sharding import bucket_bounds

    for code, es in ((_lib.DLA_F32, 4), (_lib.DLA_BF16, 2), (_lib.DLA_F64, 8)):
        for n in (0, 1, 63, 85_354, 21_296_355, 25_000_000):
            for g in (1, 2, 3, 4, 8):
                got = [_lib.shard_range(code, n, g, s) for s in range(g)]
                assert got == bucket_bounds(n, g, 256 // es)
                assert all(a * es % 256 == 0 for a, b in got if a < b)
    with pytest.raises(_lib.DlaggError):
        _lib.shard_range(_lib.DLA_F32, 10, 2, 2)


def test_result_memory_pool_reuses_blocks_only_after_release():
    """core/host_memory's pooled pageable result tensors: a block comes back only when every
    tensor on it is gone; live results never share memory; dtypes incl. bf16 keep their shape."""
    import gc

    from accdfl_amd.core import host_memory as hm

    prev = hm.result_memory()
    hm.set_result_memory("pooled")
    try:
        a = hm.result_tensor((1000, 700), torch.float32)
        b = hm.result_tensor((1000, 700), torch.float32)
        assert a.shape == (1000, 700) and a.dtype == torch.float32 and not a.is_pinned()
        assert a.data_ptr() != b.data_ptr()
        a.fill_(1.0)
        b.fill_(2.0)
        pa = a.data_ptr()
        view = a[3:5]  # a view keeps the block alive
        del a
        gc.collect()
        c = hm.result_tensor((1000, 700), torch.float32)
        assert c.data_ptr() not in (pa, b.data_ptr())
        del view
        gc.collect()
        assert hm.pool_free_bytes() >= 1000 * 700 * 4
        d = hm.result_tensor((700, 1000), torch.float32)  # same size: the released block
        assert d.data_ptr() == pa and float(b[0, 0]) == 2.0
        e = hm.result_tensor((4096, 512), torch.bfloat16)
        assert e.dtype == torch.bfloat16 and e.shape == (4096, 512)
        e.fill_(1.5)
        assert float(e.float().sum()) == 1.5 * 4096 * 512
        small = hm.result_tensor((10,), torch.float32)  # below POOL_MIN_BYTES: plain torch memory
        assert small.numel() == 10
    finally:
        hm.set_result_memory(prev)


def test_host_copy_batch_threaded_ranges(lib_path):
    """dla_host_copy_batch splits batches of 4 MiB and more into equal byte ranges over threads (a
    range may start and end inside a segment): every byte lands exactly once."""
    import numpy as np

    from accdfl_amd import _lib

    rng = np.random.default_rng(0)
    sizes = [int(x) for x in rng.integers(1, 200_000, size=400)] + [9_000_001, 0, 3]
    src = [rng.integers(0, 255, size=s, dtype=np.uint8) for s in sizes]
    dst = np.zeros(sum(sizes) + 64, dtype=np.uint8)
    offs = np.cumsum([0] + sizes[:-1])
    _lib.host_copy_batch([dst.ctypes.data + int(o) for o in offs], [a.ctypes.data for a in src], sizes)
    assert np.array_equal(dst[: sum(sizes)], np.concatenate(src)) and not dst[sum(sizes):].any()


def test_copy_pool_after_fork(lib_path):
    """dla_host_copy_batch runs large batches on a persistent thread pool; a forked child (the
    pool's threads do not exist there) must still complete its copies instead of waiting on them."""
    import numpy as np

    from accdfl_amd import _lib

    src = np.arange(6 << 20, dtype=np.uint8)   # 6 MiB: threaded
    dst = np.zeros_like(src)
    _lib.host_copy_batch([dst.ctypes.data], [src.ctypes.data], [src.nbytes])  # creates the pool
    assert np.array_equal(dst, src)
    pid = os.fork()
    if pid == 0:  # child: copy again through the (absent) pool, exit 0 on success
        code = 1
        try:
            out = np.zeros_like(src)
            _lib.host_copy_batch([out.ctypes.data], [src.ctypes.data], [src.nbytes])
            code = 0 if np.array_equal(out, src) else 2
        finally:
            os._exit(code)
    deadline = time.time() + 60
    while True:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            break
        if time.time() > deadline:
            os.kill(pid, 9)
            os.waitpid(pid, 0)
            pytest.fail("forked child hung in dla_host_copy_batch")
        time.sleep(0.05)
    assert os.WIFEXITED(status) and os.WEXITSTATUS(status) == 0


def test_numa_cpulist_and_binding_without_gpu():
    from accdfl_amd.core import host_memory

    assert host_memory._cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert host_memory._cpulist("") == set()
    if not torch.cuda.is_available():
        before = os.sched_getaffinity(0)
        assert host_memory.gpu_numa_node() is None and host_memory.bind_to_gpu_node() is None
        assert os.sched_getaffinity(0) == before


def test_copy_batch_concurrent_callers(lib_path):
    """Several host threads in dla_host_copy_batch at once (the bucket-sharded host path runs one per
    GPU): one holds the persistent pool, the others spawn their own threads; every byte lands."""
    import threading

    import numpy as np

    from accdfl_amd import _lib

    rng = np.random.default_rng(3)
    srcs = [rng.integers(0, 255, size=(9 << 20) + 7 * k, dtype=np.uint8) for k in range(6)]
    dsts = [np.zeros_like(s) for s in srcs]
    errors = []

    def work(k):
        try:
            for _ in range(5):
                dsts[k][:] = 0
                half = srcs[k].nbytes // 2
                _lib.host_copy_batch([dsts[k].ctypes.data, dsts[k].ctypes.data + half],
                                     [srcs[k].ctypes.data, srcs[k].ctypes.data + half],
                                     [half, srcs[k].nbytes - half])
                if not np.array_equal(dsts[k], srcs[k]):
                    errors.append(k)
        except Exception as exc:  # noqa: BLE001 — reported below
            errors.append(exc)

    threads = [threading.Thread(target=work, args=(k,)) for k in range(6)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in threads), "a copy hung"
    assert not errors, errors


def test_host_round_routing_and_chunks():
    """The CPU-module round sizes the host paths are chosen by (fedavg.py: _is_small, _native_chunk)."""
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    mb = 1 << 20
    assert fa._is_small(2, 341_416)                       # GL merge of two GNLeNet models
    assert fa._is_small(2, 19_729_376)                    # GL merge of two ResNet-8 models (19.7 MB rows)
    assert fa._is_small(4, 6_760_184)                     # four FEMNIST models, 27 MB
    assert not fa._is_small(4, 19_729_376)                # 79 MB: dla_host_reduce (profiles/r04s2)
    assert not fa._is_small(8, 6_760_184)                 # 54 MB: dla_host_reduce
    assert not fa._is_small(8, 19_729_376)                # 158 MB: dla_host_reduce
    assert not fa._is_small(32, 6_760_184)                # configs[2], 216 MB
    assert not fa._is_small(1, 65 * mb) and not fa._is_small(2, 0)
    for n, esize, bucket in ((8, 4, 25_000_000), (128, 2, 21_296_355), (2, 4, 4_932_344), (11, 8, 3_000_000)):
        align = 256 // esize
        c = fa._native_chunk(n, esize, bucket, align)
        assert c % align == 0 and c <= -(-bucket // align) * align
        assert n * c * esize <= fa._NATIVE_CHUNK_BYTES
        assert n * c * esize >= min(fa._NATIVE_MIN_CHUNK_BYTES, n * bucket * esize) - n * align * esize


def test_host_devices_default_is_the_current_gpu(monkeypatch):
    """A round of CPU models stays on the current GPU unless the caller opts in (the
    reference runs each peer as its own process, which must not take every GPU of the node)."""
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.delenv("ACCDFL_AMD_DEVICES", raising=False)
    cur = torch.device("cuda", 3)
    big = 1 << 34
    assert fa._devices_for(cur, big) == [cur]
    monkeypatch.setenv("ACCDFL_AMD_DEVICES", "current")
    assert fa._devices_for(cur, big) == [cur]
    monkeypatch.setenv("ACCDFL_AMD_DEVICES", "all")
    got = fa._devices_for(cur, big)
    assert got[0] == cur and sorted(d.index for d in got) == list(range(8))
    assert fa._devices_for(cur, 1 << 20) == [cur]  # too small to shard
    monkeypatch.setenv("ACCDFL_AMD_DEVICES", "2,5")
    assert fa._devices_for(cur, big) == [torch.device("cuda", 2), torch.device("cuda", 5)]
    monkeypatch.delenv("ACCDFL_AMD_DEVICES")
    fa.set_host_devices([1, 0])
    try:
        assert fa._devices_for(cur, big) == [torch.device("cuda", 1), torch.device("cuda", 0)]
    finally:
        fa.set_host_devices([])


def test_fast_parameter_walk_is_parameters():
    """fedavg._parameters (the layout passes' walk) returns exactly list(m.parameters()): order, tied
    weights and shared submodules de-duplicated, None parameters skipped; a module class with its own
    walk falls back to its parameters()."""
    from torch import nn

    from accdfl_amd.core.gradient_aggregation.fedavg import _parameters

    shared = nn.Linear(3, 3)
    m = nn.Sequential(nn.Conv2d(2, 4, 3, bias=False), nn.BatchNorm2d(4), shared,
                      nn.Sequential(shared, nn.Linear(3, 2)), nn.LSTM(3, 5, num_layers=2),
                      nn.ParameterList([nn.Parameter(torch.ones(2)), nn.Parameter(torch.zeros(3))]),
                      nn.ParameterDict({"b": nn.Parameter(torch.ones(1)), "a": nn.Parameter(torch.ones(2))}))
    m[3][1].weight = m[2].weight  # tied across submodules
    m.extra = nn.Module()
    m.extra.register_parameter("none", None)
    assert [id(p) for p in _parameters(m)] == [id(p) for p in m.parameters()]

    class OwnWalk(nn.Module):
        def __init__(self):
            super().__init__()
            self.a, self.b = nn.Linear(2, 2), nn.Linear(2, 2)

        def named_parameters(self, *args, **kw):  # reversed order: a custom walk must be honoured
            return reversed(list(super().named_parameters(*args, **kw)))

    o = nn.Sequential(nn.Linear(1, 1), OwnWalk())
    assert [id(p) for p in _parameters(o)] == [id(p) for p in o.parameters()]
    w = OwnWalk()
    assert [id(p) for p in _parameters(w)] == [id(p) for p in w.parameters()]


def test_native_walk_matches_the_python_walk():
    """csrc/walk.cpp (the host walk extension) returns the pointers of list(m.parameters()) for every
    model — tied weights and shared submodules de-duplicated, None parameters skipped — peer- or
    tensor-major, and None when the round does not qualify (shapes, dtypes, devices, density)."""
    import numpy as np
    from torch import nn

    from accdfl_amd import _lib
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    _lib.build_walk()
    _lib._walk_tried = False
    assert _lib.walk_module() is not None

    def model(seed):
        torch.manual_seed(seed)
        shared = nn.Linear(3, 3)
        m = nn.Sequential(nn.Conv2d(2, 4, 3, bias=False), nn.BatchNorm2d(4), shared,
                          nn.Sequential(shared, nn.Linear(3, 2)), nn.LSTM(3, 5),
                          nn.ParameterList([nn.Parameter(torch.ones(2))]))
        m[3][1].weight = m[2].weight
        m.extra = nn.Module()
        m.extra.register_parameter("none", None)
        return m

    models = [model(k) for k in range(5)]
    want = [[p.data_ptr() for p in m.parameters()] for m in models]
    dtype, numels, table, dev = fa._native_layout(models, -1, tensor_major=False)
    assert dtype is torch.float32 and dev == -1
    assert numels == [p.numel() for p in models[0].parameters()]
    assert np.frombuffer(table, dtype=np.uint64).tolist() == [x for row in want for x in row]
    _, _, table_t, _ = fa._native_layout(models, -1, tensor_major=True)
    assert np.frombuffer(table_t, dtype=np.uint64).reshape(len(numels), 5).T.reshape(-1).tolist() == \
        [x for row in want for x in row]
    bad = [model(9) for _ in range(2)]
    bad[1][0].weight = nn.Parameter(torch.zeros(4, 2, 3, 2))  # shape differs
    assert fa._native_layout(bad, -1, tensor_major=False) is None
    half = [model(9).half(), model(9)]  # dtype differs
    assert fa._native_layout(half, -1, tensor_major=False) is None
    strided = [model(9)]
    strided[0][0].weight = nn.Parameter(torch.zeros(4, 2, 3, 6)[..., ::2])  # not dense
    assert fa._native_layout(strided, -1, tensor_major=False) is None
    assert fa._native_layout(models, 0, tensor_major=False) is None  # CPU models asked for device 0
    # `ref`: a model outside the list sets the layout every listed model must match (a group of a round laid
    # out group by group, checked against the round's first model); its pointers are not in the table
    _, numels_r, table_r, _ = fa._native_layout(models[2:], -1, tensor_major=False, ref=models[0])
    assert numels_r == numels and np.frombuffer(table_r, dtype=np.uint64).tolist() == [x for r in want[2:] for x in r]
    assert fa._native_layout(models[1:2], -1, tensor_major=False, ref=bad[1]) is None  # shape differs from ref
    assert fa._native_layout(models[1:2], -1, tensor_major=False, ref=half[0]) is None  # dtype differs from ref
    assert fa._native_layout(bad[1:], -1, tensor_major=False, ref=bad[1]) is not None
    # tensors(): models[0]'s parameter and buffer objects in parameters() / buffers() order (the device
    # round builds the result's fresh tensors from them)
    m0 = models[0]
    m0.register_buffer("none_buf", None)
    m0.extra.register_buffer("shared_buf", m0[1].running_mean)  # the same buffer twice: listed once
    ps, bs = _lib.walk_module().tensors(m0, fa._PLAIN_SET)
    assert [id(p) for p in ps] == [id(p) for p in m0.parameters()]
    assert [id(b) for b in bs] == [id(b) for b in m0.buffers()]
    assert _lib.walk_module().tensors(m0, set()) is None  # a class outside the plain set


def test_device_round_group_schedule():
    """_group_bounds (fedavg._device_round_grouped): contiguous groups covering every model in list
    order, the first _DEVICE_GROUP_FIRST models, each later group _DEVICE_GROUP_GROWTH times the
    previous one except the last, which takes a tail shorter than its due size."""
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    f, k = fa._DEVICE_GROUP_FIRST, fa._DEVICE_GROUP_GROWTH
    if (f, k) == (16, 3):
        assert fa._group_bounds(128) == [(0, 16), (16, 64), (64, 128)]
        assert fa._group_bounds(64) == [(0, 16), (16, 64)]
    for n in range(1, 3000):
        b = fa._group_bounds(n)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
        sizes = [e - a for a, e in b]
        assert all(s > 0 for s in sizes)
        assert all(s == f * k ** i for i, s in enumerate(sizes[:-1]))
        due = f * k ** (len(sizes) - 1)
        assert sizes[-1] < 2 * due


def test_walk_memo_seeding_on_cpu():
    """walk.cpp param_views / buffer_copies store their copies straight into the deepcopy memo:
    parameters as nn.Parameter views of one allocation (offsets, strides, requires_grad kept);
    buffers copied per (device, dtype) group, skipping entries already in the memo, objects listed
    twice (one copy), storage-sharing, grad-requiring, non-contiguous and lone-in-group buffers."""
    from accdfl_amd import _lib

    mod = _lib.walk_module()
    if mod is None:
        pytest.skip("walk extension not built")
    p = [nn.Parameter(torch.randn(3, 4)), nn.Parameter(torch.randn(5), requires_grad=False)]
    flat = torch.arange(40, dtype=torch.float32)
    memo = {}
    mod.param_views(flat, p, [0, 16], memo)
    assert set(memo) == {id(x) for x in p}
    v0, v1 = memo[id(p[0])], memo[id(p[1])]
    assert type(v0) is nn.Parameter and v0.shape == (3, 4) and v0.requires_grad and not v1.requires_grad
    assert torch.equal(v0.detach().reshape(-1), flat[:12]) and torch.equal(v1.detach(), flat[16:21])
    assert v0.data_ptr() == flat.data_ptr() and v1.data_ptr() == flat.data_ptr() + 64
    # each has a storage of its own bytes (as deepcopy gives), so the reference's serialize_model
    # (pickle.dumps(state_dict())) writes each once, not the whole allocation per tensor; the
    # allocation stays alive while either does
    assert v0.untyped_storage().nbytes() == 48 and v1.untyped_storage().nbytes() == 20
    assert v0.storage_offset() == 0 and v1.storage_offset() == 0
    import pickle

    alone = pickle.dumps({"a": v0.detach().clone(), "b": v1.detach().clone()})
    assert abs(len(pickle.dumps({"a": v0.detach(), "b": v1.detach()})) - len(alone)) < 64
    del flat
    assert torch.equal(v1.detach(), torch.arange(16, 21, dtype=torch.float32))
    a, b, c = torch.randn(4), torch.randn(6), torch.arange(3)
    d = torch.arange(2)
    shared = torch.randn(8)
    view = shared[2:5]
    grad = torch.randn(3, requires_grad=True)
    strided = torch.randn(4, 4)[:, 1]
    seeded = torch.randn(2)
    bufs = [a, b, a, c, d, shared, view, grad, strided, seeded]
    memo = {id(seeded): "kept"}
    mod.buffer_copies(bufs, memo)
    assert memo[id(seeded)] == "kept"
    for x in (a, b, c, d):
        y = memo[id(x)]
        assert torch.equal(x, y) and y.dtype == x.dtype and y.data_ptr() != x.data_ptr()
    # (round 6) a fresh allocator tensor per copy, as deepcopy gives: a storage of its own at its own address
    assert [memo[id(x)].untyped_storage().nbytes() for x in (a, b, c, d)] == [16, 24, 24, 16]
    assert all(memo[id(x)].untyped_storage().data_ptr() == memo[id(x)].data_ptr() for x in (a, b, c, d))
    # param_fresh: the device round's fresh parameters, one allocator tensor each, their pointers returned
    pf = [nn.Parameter(torch.randn(3, 4)), nn.Parameter(torch.randn(5), requires_grad=False)]
    fm = {}
    ptrs = mod.param_fresh(pf, fm)
    f0, f1 = fm[id(pf[0])], fm[id(pf[1])]
    assert type(f0) is nn.Parameter and f0.shape == (3, 4) and f0.stride() == (4, 1) and f0.requires_grad
    assert not f1.requires_grad and list(ptrs) == [f0.data_ptr(), f1.data_ptr()]
    assert f0.untyped_storage().nbytes() == 48 and f0.untyped_storage().data_ptr() == f0.data_ptr()
    # param_blocks + param_wrap: the same in two halves (the blocks before the launch, the Parameters after)
    blocks, bptrs = mod.param_blocks(pf)
    assert len(blocks) == 2 and len(bptrs) == 2
    bm = {}
    mod.param_wrap(blocks, pf, bm)
    assert len(blocks) == 0  # handed over
    g0, g1 = bm[id(pf[0])], bm[id(pf[1])]
    assert type(g0) is nn.Parameter and g0.shape == (3, 4) and g0.requires_grad and not g1.requires_grad
    assert list(bptrs) == [g0.data_ptr(), g1.data_ptr()] and g0.untyped_storage().nbytes() == 48
    with pytest.raises(ValueError):
        mod.param_wrap(mod.param_blocks(pf)[0], pf[:1], {})
    import numpy as np

    pooled = torch.from_numpy(np.arange(8, dtype=np.float32))  # memory torch did not allocate
    pv = {}
    mod.param_views(pooled, [nn.Parameter(torch.zeros(3), requires_grad=False)], [2], pv)
    (pq,) = pv.values()
    assert torch.equal(pq, torch.tensor([2.0, 3.0, 4.0]))
    pq.data.resize_(5)  # resizable through the CPU allocator
    grown = memo[id(b)]
    grown.resize_(10)  # resizable like a deepcopied tensor: it moves to an allocation of its own
    assert grown.shape == (10,) and torch.equal(grown[:6], b) and torch.equal(memo[id(a)], a)
    for x in (shared, view, grad, strided):
        assert id(x) not in memo
    lone = torch.randn(2, dtype=torch.float64)
    memo = {}
    mod.buffer_copies([lone, a], memo)
    assert memo == {}  # each alone in its (device, dtype) group: left to deepcopy
