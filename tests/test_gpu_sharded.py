"""The single-process bucket-sharded reduce (dla_wsum_sharded) against the C
oracle, bit for bit.  On a one-GPU box every shard runs on GPU 0 (device ids may repeat),
which exercises the bucket split, the per-shard launches, the direct-write and gather output
modes and the event ordering; the cross-GPU (xGMI) reads run only where several GPUs are
visible (the last test).  Run on the MI355X: -m gpu."""
import numpy as np
import pytest
import torch

import golden_cases as gc
from c_oracle import c_wsum
from oracle.fedavg_oracle import same_bits

pytestmark = pytest.mark.gpu

TDT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    from accdfl_amd import _lib

    assert _lib.lib().build_id == _lib.source_build_id()
    yield


def _peers(n, numel, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(numel, generator=g) * 0.05).to(TDT[dtype]) for _ in range(n)]


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16", "f64"])
@pytest.mark.parametrize("n", [1, 8, 130])
@pytest.mark.parametrize("numel", [5, 1_000_003])
@pytest.mark.parametrize("shards", [3, 8])
@pytest.mark.parametrize("mode", ["direct", "gather"])
def test_sharded_bit_exact_on_one_gpu(dtype, n, numel, shards, mode):
    from accdfl_amd.core import wsum

    peers = _peers(n, numel, dtype, n * 31 + numel)
    w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
    want = c_wsum([gc.from_torch(p, dtype) for p in peers], w, dtype)
    dev = [p.cuda() for p in peers]
    out = wsum.wsum_sharded(dev, w, [torch.device("cuda", 0)] * shards, mode=mode)
    torch.cuda.synchronize()
    assert same_bits(gc.from_torch(out, dtype), want, dtype)


def test_allgather_gives_every_shard_the_whole_model():
    """gather=1 through the raw C ABI: every shard's own full buffer receives every bucket."""
    from accdfl_amd import _lib

    n, numel, shards = 8, 300_007, 4
    peers = _peers(n, numel, "f32", 5)
    w = [float(x) for x in np.random.default_rng(5).dirichlet(np.ones(n))]
    want = c_wsum([p.numpy() for p in peers], w, "f32")
    dev = [p.cuda() for p in peers]
    outs = [torch.full((numel,), float("nan"), device="cuda") for _ in range(shards)]
    s = torch.cuda.current_stream().cuda_stream
    _lib.wsum_sharded_ptrs(_lib.DLA_F32, [0] * shards, [p.data_ptr() for p in dev], w, numel,
                           [o.data_ptr() for o in outs], 1, [s] * shards)
    torch.cuda.synchronize()
    for o in outs:
        assert same_bits(o.cpu().numpy(), want, "f32")
    # gather=0: each buffer holds exactly its own bucket
    outs = [torch.full((numel,), float("nan"), device="cuda") for _ in range(shards)]
    _lib.wsum_sharded_ptrs(_lib.DLA_F32, [0] * shards, [p.data_ptr() for p in dev], w, numel,
                           [o.data_ptr() for o in outs], 0, [s] * shards)
    torch.cuda.synchronize()
    for r, o in enumerate(outs):
        a, b = _lib.shard_range(_lib.DLA_F32, numel, shards, r)
        host = o.cpu().numpy()
        assert same_bits(host[a:b], want[a:b], "f32")
        assert np.isnan(host[:a]).all() and np.isnan(host[b:]).all()
    _lib.shutdown()  # releases the events; the next call recreates what it needs
    out = torch.empty(numel, device="cuda")
    _lib.wsum_sharded_ptrs(_lib.DLA_F32, [0, 0], [p.data_ptr() for p in dev], w, numel, [out.data_ptr()] * 2, 0,
                           [s, s])
    torch.cuda.synchronize()
    assert same_bits(out.cpu().numpy(), want, "f32")


def test_sharded_argument_errors():
    from accdfl_amd import _lib

    s = torch.cuda.current_stream().cuda_stream
    x = torch.zeros(64, device="cuda")
    with pytest.raises(_lib.DlaggError, match="bad device id"):
        _lib.wsum_sharded_ptrs(_lib.DLA_F32, [99], [x.data_ptr()], [1.0], 64, [x.data_ptr()], 0, [s])
    with pytest.raises(_lib.DlaggError, match="gather"):
        _lib.wsum_sharded_ptrs(_lib.DLA_F32, [0], [x.data_ptr()], [1.0], 64, [x.data_ptr()], 7, [s])
    peers = [torch.zeros(64, device="cuda") for _ in range(130)]
    with pytest.raises(_lib.DlaggError, match="aliases"):  # multi-pass: out may alias peers[0] only
        _lib.wsum_sharded_ptrs(_lib.DLA_F32, [0], [p.data_ptr() for p in peers], [1.0] * 130, 64,
                               [peers[5].data_ptr()], 0, [s])


def test_fedavg_multi_device_path_bit_exact():
    """FedAvg's path for models spread over several GPUs (_reduce_multi_device), forced onto
    repeated GPU 0 here: GNLeNet shapes, every parameter reduced in place of the result."""
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    c = gc.load("gnlenet_n8_dirichlet")
    models = gc.build_models(c, "cuda:0")
    center = fa._center_copy(models[0])
    params = list(center.parameters())
    with torch.no_grad():
        fa._reduce_multi_device(params, [list(m.parameters()) for m in models], c.weights,
                                devices=[torch.device("cuda", 0)] * 3)
    torch.cuda.synchronize()
    for i, (p, want) in enumerate(zip(params, c.out)):
        assert same_bits(gc.from_torch(p, c.dtype), want, c.dtype), i


def _freed_peers_case(devs, peer_dev):
    """Peers dropped right after the sharded call and their memory reused at once on the peers'
    device: the result must still be the average of the ORIGINAL values (the peer
    device's current stream waits for the shards that read it)."""
    from accdfl_amd.core import wsum

    n, numel = 8, 4_000_037
    host = _peers(n, numel, "f32", 77)
    w = [float(x) for x in np.random.default_rng(77).dirichlet(np.ones(n))]
    want = c_wsum([p.numpy() for p in host], w, "f32")
    side = torch.cuda.Stream(peer_dev)
    with torch.cuda.stream(side):  # the caller works on a side stream of the peers' device
        peers = [p.to(peer_dev) for p in host]
        out = wsum.wsum_sharded(peers, w, devs)
        del peers
        junk = [torch.full((numel,), float("nan"), device=peer_dev) for _ in range(n)]  # reuses the blocks
    torch.cuda.synchronize()
    del junk
    assert same_bits(out.cpu().numpy(), want, "f32")


def test_sharded_peers_freed_right_after_on_one_gpu():
    _freed_peers_case([torch.device("cuda", 0)] * 3, torch.device("cuda", 0))


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (xGMI peer reads)")
def test_sharded_peers_freed_right_after_across_gpus():
    _freed_peers_case([torch.device("cuda", 0), torch.device("cuda", 1)], torch.device("cuda", 1))


@pytest.mark.parametrize("n_gpus", [2, 4, 8])
def test_models_on_several_gpus_through_fedavg(n_gpus):
    """Peers really on 2 / 4 / 8 GPUs (configs[3]'s and configs[4]'s device counts): FedAvg.aggregate
    takes the sharded multi-device path (peer access over xGMI) and matches the oracle bit for bit;
    wsum_sharded over every one of those GPUs, direct and gather."""
    if torch.cuda.device_count() < n_gpus:
        pytest.skip("needs %d GPUs (xGMI peer reads); this box has %d" % (n_gpus, torch.cuda.device_count()))
    from accdfl_amd.core import wsum
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    c = gc.load("gnlenet_n8_dirichlet")
    models = [m.to("cuda:%d" % (k % n_gpus)) for k, m in enumerate(gc.build_models(c, "cpu"))]
    out = FedAvg.aggregate(models, c.weights)
    torch.cuda.synchronize()
    for p, want in zip(out.parameters(), c.out):
        assert p.device == torch.device("cuda", 0)
        assert same_bits(gc.from_torch(p, c.dtype), want, c.dtype)
    # 64 peers (configs[3]'s count) of a ResNet-8-sized flat model spread round-robin over the GPUs
    n, numel = (8, 12_000_017) if n_gpus == 2 else (64, 4_932_344)
    peers = [t.to("cuda:%d" % (k % n_gpus)) for k, t in enumerate(_peers(n, numel, "f32", 9))]
    w = [float(x) for x in np.random.default_rng(9).dirichlet(np.ones(n))]
    want = c_wsum([p.cpu().numpy() for p in peers], w, "f32")
    devs = [torch.device("cuda", d) for d in range(n_gpus)]
    for mode in ("direct", "gather"):
        out = wsum.wsum_sharded(peers, w, devs, mode=mode)
        torch.cuda.synchronize()
        assert same_bits(out.cpu().numpy(), want, "f32"), mode


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_table_reduce_on_a_device_that_is_not_current():
    """The multi-tensor table path (>= 33 peers) for tensors on cuda:1 while device 0 is current (ADVICE
    r05): the table's upload must run on the tensors' device, through the raw call and FedAvg.aggregate."""
    from accdfl_amd.core import wsum
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    torch.cuda.set_device(0)
    d1 = torch.device("cuda", 1)
    n, numels = 40, [1000, 4099, 64, 70_001]
    g = torch.Generator().manual_seed(41)
    host = [[(torch.randn(m, generator=g) * 0.05) for _ in range(n)] for m in numels]
    w = [float(x) for x in np.random.default_rng(41).dirichlet(np.ones(n))]
    dev = [[t.to(d1) for t in row] for row in host]
    outs = [torch.empty(m, device=d1) for m in numels]
    ptrs = [t.data_ptr() for row in dev for t in row]
    wsum.wsum_multi_ptrs(torch.float32, ptrs, [o.data_ptr() for o in outs], numels, w, d1,
                         stream=torch.cuda.current_stream(d1))
    torch.cuda.synchronize(d1)
    assert torch.cuda.current_device() == 0
    for o, row in zip(outs, host):
        assert same_bits(o.cpu().numpy(), c_wsum([t.numpy() for t in row], w, "f32"), "f32")
    c = gc.load("gnlenet_n8_dirichlet")
    models = [m.to(d1) for m in gc.build_models(c, "cpu")] * 5  # 40 models: the table path
    w40 = [x / 5 for x in c.weights] * 5
    out = FedAvg.aggregate(models, w40)
    torch.cuda.synchronize(d1)
    for i, p in enumerate(out.parameters()):
        assert p.device == d1
        want = c_wsum([c.params[k % len(c.params)][i] for k in range(len(models))], w40, c.dtype)
        assert same_bits(gc.from_torch(p, c.dtype), want, c.dtype), i
