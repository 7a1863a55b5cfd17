"""Full-size parity of every BASELINE config against the C oracle (oracle/fedavg_ref.c, the
pinned restatement of accdfl/core/gradient_aggregation/fedavg.py:20-25).  Run on the MI355X:
-m gpu.  Elements are independent, so where a whole model is too large for the oracle to check
every element in seconds, the sample is chosen to cover every position inside a 16-byte chunk
(both halves of every 32-bit word of a 16-bit dtype) and every kernel region (first and last
tiles, the ragged tail).

Layouts (parameter / buffer shapes and order) come from tests/golden/layouts.json, recorded
from the reference's own ``create_model`` by tests/golden/make_layouts.py."""
import json
import os

import numpy as np
import pytest
import torch
from torch import nn

import golden_cases as gc
from c_oracle import c_wsum
from oracle.fedavg_oracle import same_bits

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TDT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}
LAYOUTS = json.load(open(os.path.join(ROOT, "tests", "golden", "layouts.json")))


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from accdfl_amd import _lib

    assert _lib.lib().build_id == _lib.source_build_id()
    yield
    torch.cuda.empty_cache()


def _slab(n, numel, dtype, seed):
    pitch = (numel + 127) // 128 * 128
    slab = torch.empty((n, pitch), dtype=TDT[dtype], device="cuda")
    for k in range(n):
        g = torch.Generator(device="cuda").manual_seed(seed + k)
        slab[k].normal_(0, 0.05, generator=g)
    return slab


def _bits(t, dtype):
    return gc.from_torch(t, dtype)


# (peers, elements, dtype): every BASELINE config's reduce at its real size — the whole model
# on one GPU and the per-GPU parameter bucket of the multi-GPU configs.
FULL = [
    pytest.param(32, 1_690_046, "f32", id="configs2_femnist_32x1690046"),
    pytest.param(64, 85_354, "f32", id="configs3_gnlenet_64x85354_whole"),
    pytest.param(64, 21_339, "f32", id="configs3_gnlenet_64x21339_bucket"),
    pytest.param(64, 4_932_344, "f32", id="configs3p_resnet8_64x4932344_whole"),
    pytest.param(64, 1_233_086, "f32", id="configs3p_resnet8_64x1233086_bucket"),
    pytest.param(128, 2_662_045, "bf16", id="configs4_speech_128x2662045_bucket"),
    pytest.param(8, 85_354, "f32", id="configs1_gnlenet_8x85354"),
]


@pytest.mark.parametrize("n,numel,dtype", FULL)
def test_config_full_size_every_element(n, numel, dtype):
    """Device-resident reduce of the whole share, compared element by element."""
    from accdfl_amd.core import wsum

    slab = _slab(n, numel, dtype, 5000 + n)
    w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
    out = wsum.wsum_rows(slab, w, numel)
    host = slab[:, :numel].cpu()
    want = c_wsum([_bits(host[k], dtype) if dtype == "bf16" else host[k].numpy() for k in range(n)], w, dtype)
    got = _bits(out, dtype) if dtype == "bf16" else out.cpu().numpy()
    assert same_bits(got, want, dtype)


def _chunk_covering_sample(numel, elems_per_chunk, seed):
    """Indices that hit every element position within a 16-byte chunk many times (an odd
    stride coprime with the chunk), plus a random set, plus the first and last 4096 elements
    (first tiles, last partial tile, ragged tail)."""
    idx = np.arange(0, numel, 61, dtype=np.int64)
    rnd = np.random.default_rng(seed).integers(0, numel, size=200_000)
    ends = np.concatenate([np.arange(0, 4096), np.arange(numel - 4096, numel)])
    idx = np.unique(np.concatenate([idx, rnd, ends]))
    assert len(set((idx % elems_per_chunk).tolist())) == elems_per_chunk
    return idx


def test_configs4_whole_model_bf16_every_lane_position():
    """configs[4] (128 peers x 21,296,355 bf16, 5.5 GB) on one GPU.  The r01 check sampled a
    stride of 64, which only ever compared the low half of word 0 of a chunk; this sample
    covers all 8 bf16 positions of a 16-byte chunk (both halves of every word)."""
    from accdfl_amd.core import wsum

    n, numel = 128, 21_296_355
    slab = _slab(n, numel, "bf16", 7)
    w = [float(x) for x in np.random.default_rng(3).dirichlet(np.ones(n))]
    out = wsum.wsum_rows(slab, w, numel)
    idx_np = _chunk_covering_sample(numel, 8, 11)
    idx = torch.from_numpy(idx_np).cuda()
    sample = slab[:, :numel].index_select(1, idx).cpu()
    want = c_wsum([_bits(sample[k].contiguous(), "bf16") for k in range(n)], w, "bf16")
    assert same_bits(_bits(out[idx], "bf16"), want, "bf16")


def _tiled(slab, n, numel, tile):
    """The PeerSlab tile-interleaved layout [n_tiles][n][tile] of the first numel elements of
    each row of a row-major slab (core/peer_slab.py; include/dlagg.h dla_wsum_slab_tiled)."""
    n_t = -(-numel // tile)
    buf = torch.zeros((n_t, n, tile), dtype=slab.dtype, device=slab.device)
    full = numel // tile
    for k in range(n):
        if full:
            buf[:full, k, :].copy_(slab[k, : full * tile].view(full, tile))
        if numel > full * tile:
            buf[full, k, : numel - full * tile].copy_(slab[k, full * tile: numel])
    return buf


def test_north_star_tiled_slab_dirichlet_every_element():
    """The headline's own kernel and layout at full size: 8 peers x 25 M fp32 in the
    tile-interleaved slab with 32 KiB tiles (what dla_slab_tile_elems picks for it), reduced by
    dla_wsum_slab_tiled with NON-uniform (Dirichlet) weights — every element against the C oracle
    (the only full-size check of this path used uniform 1/8 weights)."""
    from accdfl_amd import _lib

    n, numel = 8, 25_000_000
    tile = _lib.slab_tile_elems(_lib.DLA_F32, n, numel)
    assert tile * 4 == 32768
    slab = _slab(n, numel, "f32", 8100)
    buf = _tiled(slab, n, numel, tile)
    host = slab[:, :numel].cpu()
    del slab
    w = [float(x) for x in np.random.default_rng(81).dirichlet(np.ones(n))]
    out = torch.empty(numel, device="cuda")
    _lib.wsum_slab_tiled_ptr(_lib.DLA_F32, buf.data_ptr(), tile, n, w, numel, out.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
    want = c_wsum([host[k].numpy() for k in range(n)], w, "f32")
    assert same_bits(out.cpu().numpy(), want, "f32")


@pytest.mark.gpu
@pytest.mark.parametrize("n,dtype,tile_bytes", [
    (4, "f32", 16384), (9, "f32", 16384), (12, "f32", 16384), (16, "f32", 16384), (16, "bf16", 16384),
    (10, "bf16", 16384),
    # 32 KiB tiles: what PeerSlab uses for slabs of <= 8 rows (the GL merge N=2, small DFL rounds)
    (2, "f32", 32768), (4, "f32", 32768), (6, "f32", 32768), (8, "f32", 32768), (4, "bf16", 32768),
    (7, "bf16", 32768)])
def test_occupancy_capped_tiled_passes_every_element(n, dtype, tile_bytes):
    """The occupancy-capped launches (vec_wgs_cap: passes of 2-16 peers over >= 256 MiB of input
    get dynamic LDS so only W workgroups fit a CU) compute exactly what the uncapped kernel does: n
    peers of just over 256 MiB / n of input each, 16 and 32 KiB tiles, Dirichlet weights, a ragged
    tail of several tiles plus a partial one — every element against the C oracle."""
    from accdfl_amd import _lib

    es = 4 if dtype == "f32" else 2
    tile = tile_bytes // es
    # past the cap's 256 MiB threshold; the last 3 tiles + 12 345 elements are the ragged tail
    numel = (256 << 20) // (n * es) // tile * tile + 3 * tile + 12_345
    code = _lib.DLA_F32 if dtype == "f32" else _lib.DLA_BF16
    slab = _slab(n, numel, dtype, 9100 + n)
    buf = _tiled(slab, n, numel, tile)
    host = slab[:, :numel].cpu()
    del slab
    w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
    out = torch.empty(numel, dtype=torch.float32 if dtype == "f32" else torch.bfloat16, device="cuda")
    _lib.wsum_slab_tiled_ptr(code, buf.data_ptr(), tile, n, w, numel, out.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
    want = c_wsum([_bits(host[k], dtype) if dtype == "bf16" else host[k].numpy() for k in range(n)], w, dtype)
    got = _bits(out, dtype) if dtype == "bf16" else out.cpu().numpy()
    assert same_bits(got, want, dtype)


def test_configs4_whole_model_tiled_4k_bf16_every_lane_position():
    """configs[4]'s whole model (128 x 21,296,355 bf16) in the tile-interleaved slab with 4 KiB
    tiles (dla_slab_tile_elems for it), on the chunk-covering sample: every bf16 position of a
    chunk, the first and last tiles and the ragged tail."""
    from accdfl_amd import _lib

    n, numel = 128, 21_296_355
    tile = _lib.slab_tile_elems(_lib.DLA_BF16, n, numel)
    assert tile * 2 == 4096
    slab = _slab(n, numel, "bf16", 1300)
    buf = _tiled(slab, n, numel, tile)
    idx_np = _chunk_covering_sample(numel, 8, 13)
    idx = torch.from_numpy(idx_np).cuda()
    sample = slab[:, :numel].index_select(1, idx).cpu()
    del slab
    w = [float(x) for x in np.random.default_rng(128).dirichlet(np.ones(n))]
    out = torch.empty(numel, dtype=torch.bfloat16, device="cuda")
    _lib.wsum_slab_tiled_ptr(_lib.DLA_BF16, buf.data_ptr(), tile, n, w, numel, out.data_ptr(),
                             torch.cuda.current_stream().cuda_stream)
    want = c_wsum([_bits(sample[k].contiguous(), "bf16") for k in range(n)], w, "bf16")
    assert same_bits(_bits(out[idx], "bf16"), want, "bf16")


class _LayoutModel(nn.Module):
    """A module with a reference model's parameter and buffer layout (names flattened)."""

    def __init__(self, lay, dtype, seed):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.ps = nn.ParameterList([nn.Parameter((torch.randn(s, generator=g) * 0.05).to(dtype))
                                    for _, s, _ in lay["params"]])
        for j, (_, s, bdt) in enumerate(lay["buffers"]):
            if bdt == "int64":
                self.register_buffer("b%d" % j, torch.full(s, seed, dtype=torch.int64))
            else:
                self.register_buffer("b%d" % j, torch.randn(s, generator=g).to(getattr(torch, bdt)))


@pytest.mark.parametrize("placement", ["cpu", "cuda:0"])
def test_resnet34_layout_through_fedavg_aggregate(placement):
    """google_speech ResNet-34 (110 parameter tensors + 108 BN buffers, 21,296,355 params)
    in bf16, 16 peers, through the drop-in FedAvg.aggregate with CPU modules (host-staged path)
    and device modules (multi-tensor kernel).  Every parameter element is compared with the
    oracle; buffers are models[0]'s (fedavg.py:20), never averaged."""
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    lay = LAYOUTS["google_speech_resnet34"]
    assert len(lay["params"]) == 110 and lay["n_params"] == 21_296_355
    n = 16
    models = [_LayoutModel(lay, torch.bfloat16, 300 + k).to(placement) for k in range(n)]
    w = [float(x) for x in np.random.default_rng(16).dirichlet(np.ones(n))]
    out = FedAvg.aggregate(models, w)
    torch.cuda.synchronize()
    flat = [torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu() for m in models]
    want = c_wsum([_bits(f, "bf16") for f in flat], w, "bf16")
    got = _bits(torch.cat([p.detach().reshape(-1) for p in out.parameters()]), "bf16")
    assert same_bits(got, want, "bf16")
    assert all(p.device.type == torch.device(placement).type for p in out.parameters())
    assert all(p.requires_grad for p in out.parameters())
    for b, b0 in zip(out.buffers(), models[0].buffers()):
        assert b.dtype == b0.dtype and torch.equal(b.cpu(), b0.cpu())


@pytest.mark.parametrize("name,n,dtype", [("cifar10_resnet8", 64, "f32"), ("femnist_cnn", 32, "f32"),
                                          ("cifar10_resnet8", 2, "f32"), ("cifar10_resnet8", 4, "f32"),
                                          ("femnist_cnn", 8, "f32")])
def test_config_layouts_through_fedavg_aggregate(name, n, dtype):
    """configs[3'] ResNet-8 (64 peers, 32 tensors, 4.93 M params) and configs[2] FEMNIST CNN
    (32 peers, 8 tensors, 1.69 M params) through FedAvg.aggregate on CPU modules (dla_host_reduce),
    and the GL-merge-sized rounds of the same layouts (2-8 peers: the small-round path below 48 MiB,
    with 19.7 MB rows, dla_host_reduce above), every element against the oracle."""
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    lay = LAYOUTS[name]
    models = [_LayoutModel(lay, TDT[dtype], 900 + k) for k in range(n)]
    w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
    out = FedAvg.aggregate(models, w)
    flat = [torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy() for m in models]
    want = c_wsum(flat, w, dtype)
    got = torch.cat([p.detach().reshape(-1) for p in out.parameters()]).numpy()
    assert same_bits(got, want, dtype)
    for b, b0 in zip(out.buffers(), models[0].buffers()):
        assert torch.equal(b, b0)
