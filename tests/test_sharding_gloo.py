"""Multi-rank sharding logic on CPU (gloo, world_size 2, 3 and 8), fp32 and bf16:
bucket-sharded and peer-sharded (all-to-all transpose) FedAvg reassemble to exactly the
single-process C-oracle result (fedavg.py:20-25 over the whole model).  The per-bucket
reduce is the NumPy oracle injected as the reducer on CPU, and the libdlagg kernel on the
box's one GPU (every rank sharing cuda:0) for the -m gpu cases; this exercises the
exchange steps, the bucket alignment of each dtype (64 fp32 / 128 bf16 elements), ragged
and empty trailing buckets, and 128 / 130 peers (one and two kernel passes)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

_TORCH = {"f32": torch.float32, "bf16": torch.bfloat16}
_BITS = {"f32": (np.uint32, torch.int32), "bf16": (np.uint16, torch.int16)}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _to_bits(t: torch.Tensor, dtype: str) -> np.ndarray:
    """Raw bit patterns of a f32 / bf16 tensor (uint32 / uint16)."""
    np_u, t_i = _BITS[dtype]
    return t.contiguous().cpu().view(t_i).numpy().view(np_u).copy()


def _from_bits(bits: np.ndarray, dtype: str) -> torch.Tensor:
    np_u, t_i = _BITS[dtype]
    signed = np.int32 if np_u is np.uint32 else np.int16
    return torch.from_numpy(np.ascontiguousarray(bits).view(signed)).view(_TORCH[dtype])


def _oracle_reducer(dtype):
    def red(peers, weights, out):
        from oracle.fedavg_oracle import fedavg_bits

        res = fedavg_bits([_to_bits(p, dtype) if dtype == "bf16" else p.numpy() for p in peers], weights, dtype)
        out.copy_(_from_bits(res.view(_BITS[dtype][0]), dtype))
        return out
    return red


def _hip_reducer(peers, weights, out):
    """The libdlagg kernel on cuda:0 (every rank of the rehearsal shares the one GPU)."""
    from accdfl_amd.core import wsum

    dev = torch.device("cuda", 0)
    out.copy_(wsum.wsum([p.to(dev) for p in peers], weights).cpu())
    return out


def _inputs(n_peers, n_elems, dtype="f32"):
    """Seeded peers as bit patterns (fp32 values, bf16 = the RNE cast of the same values)
    and Dirichlet weights as Python floats."""
    rng = np.random.default_rng(123)
    vals = (rng.standard_normal((n_peers, n_elems), dtype=np.float32) * np.float32(0.05))
    weights = [float(x) for x in rng.dirichlet(np.ones(n_peers))]
    if dtype == "f32":
        return vals.view(np.uint32), weights
    return _to_bits(torch.from_numpy(vals).to(torch.bfloat16), "bf16"), weights


def _worker(rank, world, port, n_peers, n_elems, root, q, reducer="oracle", dtype="f32"):
    import sys

    for p in (os.path.join(root, "decentralized-learning_amd"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.set_num_threads(1)
    nccl = reducer == "nccl"
    dev = torch.device("cuda", rank) if nccl else torch.device("cpu")
    if nccl:
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from accdfl_amd.core import wsum
        from accdfl_amd.core.sharding import BucketShardedFedAvg

        bits, weights = _inputs(n_peers, n_elems, dtype)
        peers = _from_bits(bits, dtype)
        red = {"hip": _hip_reducer, "oracle": _oracle_reducer(dtype),
               "nccl": lambda ps, w, out: wsum.wsum(list(ps), w, out=out)}[reducer]
        sh = BucketShardedFedAvg(n_elems, _TORCH[dtype], device=dev, reducer=red)
        # (1) bucket-sharded: this rank holds its bucket of every peer, zero-padded to bucket_len
        s, e = sh.local_range
        padded = torch.zeros((n_peers, sh.bucket_len), dtype=_TORCH[dtype])
        padded[:, : e - s] = peers[:, s:e]
        full = sh.all_gather(sh.reduce_bucket(list(padded.to(dev)), weights))
        res = {"bucket": _to_bits(full, dtype), "range": (s, e), "bucket_len": sh.bucket_len}
        if n_peers % world == 0:
            # (2) peer-sharded: rank r holds whole peers r*m .. r*m+m-1
            m = n_peers // world
            local = peers[rank * m:(rank + 1) * m].contiguous().to(dev)
            res["peer"] = _to_bits(sh.aggregate_peer_sharded(local, weights), dtype)
            if dtype == "f32":
                res["rs"] = sh.aggregate_peer_sharded(local, weights, exact=False).cpu().numpy().copy()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


# world, peers, elements, dtype: ragged last buckets (10_001 / 4_099), every bucket but the first
# empty (37 over 2 and 8 ranks), bf16's 128-element alignment, 8 ranks with 128 peers (one kernel
# pass) and 130 peers (two passes; no peer-sharded split: 130 is not a multiple of 8)
_CPU_CASES = [(2, 8, 10_001, "f32"), (3, 6, 4_099, "f32"), (2, 4, 37, "f32"),
              (2, 8, 10_001, "bf16"), (3, 6, 4_099, "bf16"), (8, 4, 37, "bf16"),
              (8, 128, 2_051, "bf16"), (8, 130, 1_031, "f32")]


@pytest.mark.parametrize("world,n_peers,n_elems,dtype", _CPU_CASES)
def test_sharded_fedavg_is_bit_exact(world, n_peers, n_elems, dtype):
    _run_sharded(world, n_peers, n_elems, "oracle", dtype)


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_peers,n_elems,dtype", [
    (2, 8, 1_000_003, "f32"), (4, 8, 65_537, "f32"), (2, 8, 1_000_003, "bf16"),
    # configs[4]'s split: 8 ranks, bf16, 128 peers (one pass) and 130 (two passes), ragged last bucket
    (8, 128, 1_000_003, "bf16"), (8, 130, 262_147, "bf16"), (8, 128, 262_147, "f32")])
def test_sharded_fedavg_hip_reducer_is_bit_exact(world, n_peers, n_elems, dtype):
    """The same exchange steps with the libdlagg kernel as each rank's bucket reducer
    (gloo ranks sharing the box's one GPU; the RCCL transport is the driver's 8-GPU run)."""
    _run_sharded(world, n_peers, n_elems, "hip", dtype)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="RCCL needs one GPU per rank (the driver's multi-GPU node)")
@pytest.mark.parametrize("world,n_peers,n_elems,dtype", [(2, 8, 1_000_003, "f32"), (2, 8, 1_000_003, "bf16")])
def test_sharded_fedavg_over_rccl(world, n_peers, n_elems, dtype):
    """The same exchange steps over RCCL (backend "nccl"), one GPU per rank, device tensors:
    all-gather and all-to-all bit-exact, reduce-scatter within its stated bound."""
    if world > torch.cuda.device_count():
        pytest.skip("needs %d GPUs" % world)
    _run_sharded(world, n_peers, n_elems, "nccl", dtype)


def _hashed_rows(peers, a, b, dtype, chunk=1 << 18):
    """Peers ``peers``' elements [a, b) of a synthetic model whose every element is a hash of (peer,
    index): any rank builds any slice of any peer without generating whole rows (configs[4]'s 128 x
    21.3 M bf16 model would be 5.4 GB per rank).  Values: uniform in +-0.05 scaled by 2^-0..-7, the
    bf16 form the RNE cast of the f32 one.  Returns a CPU tensor [len(peers), b - a]."""
    peers = np.asarray(list(peers), dtype=np.uint64)
    out = torch.empty((len(peers), max(0, b - a)), dtype=_TORCH[dtype])
    with np.errstate(over="ignore"):
        for c0 in range(a, b, chunk):
            c1 = min(b, c0 + chunk)
            x = (np.arange(c0, c1, dtype=np.uint64)[None, :] * np.uint64(0x9E3779B97F4A7C15)
                 + (peers[:, None] + np.uint64(1)) * np.uint64(0xD1B54A32D192ED03))
            x ^= x >> np.uint64(31)
            x *= np.uint64(0xBF58476D1CE4E5B9)
            x ^= x >> np.uint64(29)
            u = ((x >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24) - np.float32(0.5)) * np.float32(0.1)
            u *= np.exp2(-((x >> np.uint64(13)) & np.uint64(7)).astype(np.float32))
            out[:, c0 - a:c1 - a] = torch.from_numpy(u).to(_TORCH[dtype])
    return out


def _rccl_worker(rank, world, port, n_peers, n_elems, root, q, dtype, backend="nccl"):
    """One rank of a full-size RCCL case: builds its bucket of every peer and its own whole peers, runs
    the bucket-sharded all-gather, the exact all-to-all and (f32) the reduce-scatter mode, and checks ITS
    bucket of each gathered result against the C oracle over the same bucket; the parent checks that every
    rank gathered the same bytes (sha256), so every bucket of every rank's result is oracle-checked.
    backend "gloo": the same steps on CPU tensors with the NumPy oracle as the reducer (CPU rehearsal)."""
    import hashlib
    import sys

    for p in (os.path.join(root, "decentralized-learning_amd"), root, os.path.join(root, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.set_num_threads(2)
    if backend == "nccl":
        dev = torch.device("cuda", rank)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:  # "gloo": CPU tensors, the oracle reducer; "gloo-hip": CPU tensors, the libdlagg reducer on cuda:0
        dev = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from c_oracle import c_wsum
        from accdfl_amd.core.sharding import BucketShardedFedAvg

        weights = [float(x) for x in np.random.default_rng(n_peers).dirichlet(np.ones(n_peers))]
        # RCCL: the libdlagg reducer (the sharding module's default)
        sh = BucketShardedFedAvg(n_elems, _TORCH[dtype], device=dev,
                                 reducer={"nccl": None, "gloo": _oracle_reducer(dtype), "gloo-hip": _hip_reducer}[backend])
        s, e = sh.local_range
        mine = _hashed_rows(range(n_peers), s, e, dtype)
        want = c_wsum(list(_to_bits(mine, dtype)) if dtype == "bf16" else list(mine.numpy()), weights, dtype)
        want = want.view(_BITS[dtype][0])
        padded = torch.zeros((n_peers, sh.bucket_len), dtype=_TORCH[dtype], device=dev)
        padded[:, : e - s] = mine.to(dev)
        full = sh.all_gather(sh.reduce_bucket(list(padded), weights))
        del padded
        res = {"range": (s, e)}

        def check(name, t):
            bits = _to_bits(t, dtype)
            res[name + "_ok"] = bool(np.array_equal(bits[s:e], want)) and bits.size == n_elems
            res[name + "_sha"] = hashlib.sha256(bits.tobytes()).hexdigest()

        check("bucket", full)
        m = n_peers // world
        local = _hashed_rows(range(rank * m, (rank + 1) * m), 0, n_elems, dtype).to(dev)
        check("peer", sh.aggregate_peer_sharded(local, weights))
        if dtype == "f32":
            rs = sh.aggregate_peer_sharded(local, weights, exact=False).cpu().numpy()[s:e].astype(np.float64)
            vals = mine.numpy().astype(np.float64)
            bound = n_peers * 2.0 ** -23 * np.sum(np.abs(np.asarray(weights)[:, None] * vals), axis=0)
            err = np.abs(rs - want.view(np.float32).astype(np.float64))
            res["rs_ok"] = bool(np.all(err <= bound + 1e-45))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


# BASELINE configs[3] (64 peers over 4 GPUs; ResNet-8's 4 932 344 f32 parameters: each rank's bucket is
# configs[3']'s 1 233 086-element share) and configs[4] (128 google_speech ResNet-34 models, 21 296 355
# bf16 parameters, over 8 GPUs: 2 662 144 elements per rank)
@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,n_peers,n_elems,dtype", [(4, 64, 4_932_344, "f32"), (8, 128, 21_296_355, "bf16")])
def test_sharded_fedavg_over_rccl_at_config_size(world, n_peers, n_elems, dtype):
    """configs[3] and configs[4]'s own splits over RCCL at full model size: all-gather and all-to-all
    bit-exact against the C oracle bucket by bucket, reduce-scatter within its stated bound."""
    if not torch.cuda.is_available() or torch.cuda.device_count() < world:
        pytest.skip("needs %d GPUs (one per rank, RCCL over xGMI); this box has %d"
                    % (world, torch.cuda.device_count() if torch.cuda.is_available() else 0))
    _run_config_split(world, n_peers, n_elems, dtype, "nccl")


@pytest.mark.parametrize("world,n_peers,n_elems,dtype", [(4, 64, 40_009, "f32"), (8, 128, 21_297, "bf16")])
def test_config_split_rehearsal_on_cpu(world, n_peers, n_elems, dtype):
    """The full-size RCCL cases' worker, its per-rank oracle check and the digest agreement, rehearsed
    over gloo on the CPU at the same world sizes and peer counts (1/500 and 1/1000 of the elements)."""
    _run_config_split(world, n_peers, n_elems, dtype, "gloo")


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,n_peers,n_elems,dtype", [(4, 64, 4_932_344, "f32"), (8, 128, 21_296_355, "bf16")])
def test_config_split_full_size_hip_reducer_over_gloo(world, n_peers, n_elems, dtype):
    """configs[3] and configs[4]'s splits at FULL model size on the one-GPU box: the same ranks, exchanges
    and per-rank oracle check as the RCCL case, the collectives over gloo and every rank's bucket reduced by
    the libdlagg kernel on the box's one GPU (the 8-rank HIP-reducer cases ran 1 M
    elements per model, not configs[4]'s 21 296 355)."""
    _run_config_split(world, n_peers, n_elems, dtype, "gloo-hip")


def _run_config_split(world, n_peers, n_elems, dtype, backend):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rccl_worker, args=(r, world, port, n_peers, n_elems, root, q, dtype, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = dict(q.get(timeout=600) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert sum(r["range"][1] - r["range"][0] for r in results.values()) == n_elems
    for name in ("bucket", "peer"):
        assert all(r[name + "_ok"] for r in results.values()), (name, {k: r[name + "_ok"] for k, r in results.items()})
        assert len({r[name + "_sha"] for r in results.values()}) == 1, name
    assert results[0]["bucket_sha"] == results[0]["peer_sha"]
    if dtype == "f32":
        assert all(r["rs_ok"] for r in results.values())


def test_hashed_rows_slices_agree():
    """_hashed_rows: a slice built alone equals the same slice of the whole rows (what lets every rank of
    the full-size RCCL cases build only its bucket)."""
    whole = _hashed_rows(range(5), 0, 1000, "bf16", chunk=128)
    assert torch.equal(_hashed_rows([1, 3], 300, 777, "bf16"), whole[[1, 3], 300:777])
    f = _hashed_rows(range(3), 0, 4096, "f32")
    assert f.abs().max() <= 0.05 and f.std() > 0.001 and len(set(f[0].tolist())) > 4000


def test_reduce_scatter_mode_is_fp32_fp64_only():
    """exact=False (reduce-scatter, re-associated) states its bound for fp32 / fp64 sums only."""
    from accdfl_amd.core.sharding import BucketShardedFedAvg

    sh = BucketShardedFedAvg(64, torch.bfloat16, reducer=_oracle_reducer("bf16"))
    with pytest.raises(ValueError, match="float32 / float64 only"):
        sh.aggregate_peer_sharded(torch.zeros((2, 64), dtype=torch.bfloat16), exact=False)


def test_bucket_alignment_per_dtype():
    """Bucket starts are 256-byte aligned: 64 fp32 / 128 bf16 elements; trailing buckets may be empty."""
    from accdfl_amd.core.sharding import BucketShardedFedAvg, bucket_bounds

    assert bucket_bounds(1_000_003, 8, 128)[-1] == (7 * 125_056, 1_000_003)
    assert bucket_bounds(37, 8, 128) == [(0, 37)] + [(37, 37)] * 7
    for dt, align in ((torch.float32, 64), (torch.bfloat16, 128), (torch.float64, 32)):
        sh = BucketShardedFedAvg(21_296_355, dt, reducer=_oracle_reducer("f32"))
        assert all(s % align == 0 for s, _ in sh.bounds)
        assert sh.bounds[-1][1] == 21_296_355


def _run_sharded(world, n_peers, n_elems, reducer, dtype="f32"):
    from c_oracle import c_wsum

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_peers, n_elems, root, q, reducer, dtype))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = [q.get(timeout=300) for _ in range(world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    bits, weights = _inputs(n_peers, n_elems, dtype)
    peers = list(bits) if dtype == "bf16" else list(bits.view(np.float32))
    want = c_wsum(peers, weights, dtype).view(_BITS[dtype][0])
    covered = 0
    for rank, res in sorted(results, key=lambda r: r[0]):
        s, e = res["range"]
        covered += e - s
        assert np.array_equal(res["bucket"], want), "bucket-sharded rank %d (%s)" % (rank, dtype)
        if "peer" in res:
            assert np.array_equal(res["peer"], want), "peer-sharded rank %d (%s)" % (rank, dtype)
        if "rs" in res:
            # tolerance of the reduce-scatter (re-associating) mode: N * 2^-23 * sum_k |w_k p_k|
            vals = bits.view(np.float32).astype(np.float64)
            bound = n_peers * 2.0 ** -23 * np.sum(np.abs(np.asarray(weights)[:, None] * vals), axis=0)
            err = np.abs(res["rs"].astype(np.float64) - want.view(np.float32).astype(np.float64))
            assert np.all(err <= bound + 1e-45), "reduce-scatter mode rank %d: max err %g" % (rank, err.max())
    assert covered == n_elems


def test_bucket_bounds_properties_fuzz():
    """bucket_bounds over 2 000 seeded (n_elems, world, alignment) draws: the buckets tile [0, n_elems)
    in rank order with no gap or overlap, every non-empty bucket starts on the alignment, and no
    bucket exceeds the ceil-divided, aligned share."""
    from accdfl_amd.core.sharding import bucket_bounds

    rng = np.random.default_rng(11)
    for _ in range(2000):
        n = int(rng.choice([0, 1, 7, 63, 64, 65, 1000, 4099, 21_296_355, int(rng.integers(0, 1 << 26))]))
        world = int(rng.integers(1, 17))
        align = int(rng.choice([1, 16, 32, 64, 128]))
        b = bucket_bounds(n, world, align)
        assert len(b) == world
        assert b[0][0] == 0 and b[-1][1] == n
        for (s0, e0), (s1, e1) in zip(b, b[1:]):
            assert e0 == s1 and s0 <= e0
        share = -(-(-(-n // world) if n else 0) // align) * align
        for s, e in b:
            assert s <= e and e - s <= share
            assert s == e or s % align == 0


def _random_sharding_cases(k=4, seed=29):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(k):
        world = int(rng.choice([2, 3, 4, 5, 8]))
        n_peers = int(rng.choice([3, 7, 16, 40, 128, 130]))
        out.append((world, n_peers, int(rng.integers(1, 300_000)), str(rng.choice(["f32", "bf16"]))))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_peers,n_elems,dtype", _random_sharding_cases())
def test_sharded_fedavg_hip_reducer_random_shapes(world, n_peers, n_elems, dtype):
    """Seeded random world sizes, peer counts and lengths (ragged and empty trailing buckets, one and two
    kernel passes) through the bucket-sharded and peer-sharded exchanges with the libdlagg reducer."""
    _run_sharded(world, n_peers, n_elems, "hip", dtype)


@pytest.mark.parametrize("world,n_peers,n_elems,dtype", _random_sharding_cases(k=2, seed=31))
def test_sharded_fedavg_random_shapes(world, n_peers, n_elems, dtype):
    """The same seeded random shapes on the CPU (the NumPy oracle as each rank's bucket reducer)."""
    _run_sharded(world, n_peers, min(n_elems, 50_000), "oracle", dtype)
