"""Multi-rank sharding logic on CPU (gloo, world_size 2 and 3): bucket-sharded and
peer-sharded (all-to-all transpose) FedAvg reassemble to exactly the single-process
oracle result.  The per-bucket reduce is the CPU oracle injected as the reducer —
the kernel itself is covered by the -m gpu tests; this exercises the exchange steps."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_reducer(peers, weights, out):
    from oracle.fedavg_oracle import fedavg_bits

    res = fedavg_bits([p.numpy() for p in peers], weights, "f32")
    out.copy_(torch.from_numpy(res))
    return out


def _hip_reducer(peers, weights, out):
    """The libdlagg kernel on cuda:0 (every rank of the rehearsal shares the one GPU)."""
    from accdfl_amd.core import wsum

    dev = torch.device("cuda", 0)
    out.copy_(wsum.wsum([p.to(dev) for p in peers], weights).cpu())
    return out


def _inputs(n_peers, n_elems):
    rng = np.random.default_rng(123)
    peers = (rng.standard_normal((n_peers, n_elems)) * 0.05).astype(np.float32)
    weights = [float(x) for x in rng.dirichlet(np.ones(n_peers))]
    return peers, weights


def _worker(rank, world, port, n_peers, n_elems, root, q, reducer="oracle"):
    import sys

    for p in (os.path.join(root, "decentralized-learning_amd"), root):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
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

        peers, weights = _inputs(n_peers, n_elems)
        red = {"hip": _hip_reducer, "oracle": _oracle_reducer,
               "nccl": lambda ps, w, out: wsum.wsum(list(ps), w, out=out)}[reducer]
        sh = BucketShardedFedAvg(n_elems, torch.float32, device=dev, reducer=red)
        # (1) bucket-sharded: this rank holds its bucket of every peer
        s, e = sh.local_range
        buckets = [torch.from_numpy(peers[k, s:e].copy()) for k in range(n_peers)]
        padded = [torch.cat([b, torch.zeros(sh.bucket_len - b.numel())]).to(dev) for b in buckets]
        full = sh.all_gather(sh.reduce_bucket(padded, weights))
        # (2) peer-sharded: rank r holds whole peers r*m .. r*m+m-1
        m = n_peers // world
        local = torch.from_numpy(peers[rank * m:(rank + 1) * m].copy()).to(dev)
        full2 = sh.aggregate_peer_sharded(local, weights)
        full3 = sh.aggregate_peer_sharded(local, weights, exact=False)
        q.put((rank, full.cpu().numpy().view(np.uint32).copy(), full2.cpu().numpy().view(np.uint32).copy(),
               full3.cpu().numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_peers,n_elems", [(2, 8, 10_001), (3, 6, 4_099), (2, 4, 37)])
def test_sharded_fedavg_is_bit_exact(world, n_peers, n_elems):
    _run_sharded(world, n_peers, n_elems, "oracle")


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_peers,n_elems", [(2, 8, 1_000_003), (4, 8, 65_537)])
def test_sharded_fedavg_hip_reducer_is_bit_exact(world, n_peers, n_elems):
    """The same exchange steps with the libdlagg kernel as each rank's bucket reducer
    (gloo ranks sharing the box's one GPU; the RCCL transport is the driver's 8-GPU run)."""
    _run_sharded(world, n_peers, n_elems, "hip")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="RCCL needs one GPU per rank (the driver's multi-GPU node)")
@pytest.mark.parametrize("world,n_peers,n_elems", [(2, 8, 1_000_003)])
def test_sharded_fedavg_over_rccl(world, n_peers, n_elems):
    """The same exchange steps over RCCL (backend "nccl"), one GPU per rank, device tensors:
    all-gather and all-to-all bit-exact, reduce-scatter within its stated bound."""
    _run_sharded(world, n_peers, n_elems, "nccl")


def test_reduce_scatter_mode_is_fp32_fp64_only():
    """exact=False (reduce-scatter, re-associated) states its bound for fp32 / fp64 sums only."""
    from accdfl_amd.core.sharding import BucketShardedFedAvg

    sh = BucketShardedFedAvg(64, torch.bfloat16, reducer=_oracle_reducer)
    with pytest.raises(ValueError, match="float32 / float64 only"):
        sh.aggregate_peer_sharded(torch.zeros((2, 64), dtype=torch.bfloat16), exact=False)


def _run_sharded(world, n_peers, n_elems, reducer):
    from oracle.fedavg_oracle import fedavg_bits

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_peers, n_elems, root, q, reducer))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    peers, weights = _inputs(n_peers, n_elems)
    want = fedavg_bits(list(peers), weights, "f32").view(np.uint32)
    # tolerance of the reduce-scatter (re-associating) mode: N * 2^-23 * sum_k |w_k p_k|
    bound = n_peers * 2.0 ** -23 * np.sum(np.abs(np.asarray(weights)[:, None] * peers.astype(np.float64)), axis=0)
    for rank, full, full2, full3 in results:
        assert np.array_equal(full, want), "bucket-sharded rank %d" % rank
        assert np.array_equal(full2, want), "peer-sharded rank %d" % rank
        err = np.abs(full3.astype(np.float64) - want.view(np.float32).astype(np.float64))
        assert np.all(err <= bound + 1e-45), "reduce-scatter mode rank %d: max err %g" % (rank, err.max())
