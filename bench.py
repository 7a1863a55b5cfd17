"""Benchmark of the accdfl FedAvg aggregation reduce on MI355X.

Metric (BASELINE.json): aggregated-model GB/s (device-resident), N-peer reduce.
Workload per GPU (north star, BASELINE.json north_star): 8 peers x 25,000,000 fp32
parameters, inputs resident in HBM.  With --gpus G (one process per GPU, launched by
torch.distributed.run) the model is G x 25 M parameters, bucket-sharded: every rank
reduces its own 25 M-parameter bucket of all 8 peers (weak scaling, no data-path
collective; the optional all-gather that reassembles the model is timed separately).

One step = one launch of the libdlagg kernel over one rank's bucket.
Algorithmic bytes per step per rank = (N + 1) * P * 4 (N peer reads + 1 output write).
value = sum over ranks of bytes / max-over-ranks step time.

Launch: under torch.distributed.run (WORLD_SIZE set) every process is one rank.  Without
it, ``--gpus G`` (G > 1) makes this process start G ranks itself through
torch.distributed.run before anything touches a GPU, and wait for them; every rank then
checks that the process group really has G ranks.

Extra objects on the JSON line:
  roofline      dominant kernel (the headline launch's): achieved GB/s from HIP events on the
                launch stream over the timed region vs 8 TB/s HBM peak; traffic = PMC HBM
                bytes per launch from profiles/pmc_traffic.json (null if not collected)
  separate_buffers  the same peers as one buffer per peer (what FedAvg.aggregate on device
                modules reduces) — the row-major comparison to the PeerSlab layout
  launch        backend, world size and who started the ranks (rank-count check)
  strong_scaling  ("scaling": "strong") FIXED models — the north-star 8 x 25 M fp32 model,
                configs[3] / configs[3'] (64 peers) and configs[4] (128 peers, bf16) — each
                split into N parameter buckets, one per rank: whole-model bytes / max-over-ranks
                step time, inputs rotated so the working set exceeds the 256 MiB Infinity
                Cache; the RCCL all-gather that reassembles the model is timed on its own
  collectives   (N > 1) the RCCL legs: all-gather reassembly, exact peer-sharded
                all-to-all path, reduce-scatter tolerance path
  host_inclusive_sharded  (N > 1, rank 0) the CPU-module path bucket-sharded over GPUs
                0..N-1 of one process (each bucket over its own PCIe link)
  baseline_configs  (N = 1) every BASELINE config at its per-GPU share, staged as PeerSlab
                holds it (prepared launch)
  host_inclusive, host_inclusive_small, wire_ingress, dfl_round  (N = 1) FedAvg.aggregate on
                CPU modules (PCIe-inclusive), the GNLeNet small rounds, one peer's wire bytes
                into HBM, one DFL round from EVA blocks to outgoing bytes
  host_inclusive_configs  (N = 1) every GPU config's whole model as CPU modules with the reference's
                real layout (tests/golden/layouts.json) through FedAvg.aggregate, pageable and
                page-locked peers
  cpu_baseline  (N = 1, rank 0) the reference's torch-CPU op sequence (oracle/fedavg_oracle.py,
                kind "port") on this host's CPU share, bounded sample, product temporary held
                (value), and the literal sequence in a fresh process (cold_fresh_process); every
                other CPU comparison (per config, the config layouts, GNLeNet rounds, the
                reference-style DFL round) is timed in this leg too, the only one that runs the
                oracle port
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import socket
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "aggregated-model GB/s (device-resident), N-peer reduce; 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md)
NS_PEERS = 8
NS_PARAMS = 25_000_000
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")

# Every BASELINE.json config as the share ONE GPU reduces: name ->
# (peers, params of the whole model, dtype, GPUs the config names).  A G-GPU config's
# per-GPU share is its parameter bucket: params / G of every peer.
CONFIGS = {
    "configs[0] spambase LinearModel, 4 peers (CPU plumbing in the reference)": (4, 116, "f32", 1),
    "configs[1] CIFAR-10 GNLeNet, 8 peers, 1 GPU": (8, 85_354, "f32", 1),
    "configs[2] FEMNIST CNN, 32 peers, 1 GPU": (32, 1_690_046, "f32", 1),
    # configs[3] names 4 GPUs, but its whole model is 22 MB: below the product's sharding threshold
    # (fedavg._MIN_SHARD_BYTES per GPU), so the product reduces it on one GPU — that is the line
    "configs[3] CIFAR-10 GNLeNet, 64 peers, whole model on 1 GPU (not sharded: 22 MB)": (64, 85_354, "f32", 1),
    "configs[3'] CIFAR-10 ResNet-8 variant, 64 peers, 4 GPUs (per-GPU bucket)": (64, 4_932_344, "f32", 4),
    "configs[4] google_speech ResNet-34, 128 peers, bf16, 8 GPUs (per-GPU bucket)": (128, 21_296_355, "bf16", 8),
    "configs[4] google_speech ResNet-34, 128 peers, bf16, whole model on 1 GPU": (128, 21_296_355, "bf16", 1),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--peers", type=int, default=NS_PEERS)
    ap.add_argument("--params", type=int, default=NS_PARAMS)
    ap.add_argument("--dtype", default="f32", choices=["f32", "bf16", "f16", "f64"])
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--chunks", type=int, default=0)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--no-small", action="store_true")
    ap.add_argument("--coll-params", type=int, default=0, help="params per rank bucket for the RCCL legs")
    ap.add_argument("--no-collectives", action="store_true",
                    help="skip the RCCL legs (all-gather, peer-sharded all-to-all / reduce-scatter) at N > 1")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) for real runs; gloo only to rehearse "
                                                             "several ranks on one GPU")
    ap.add_argument("--no-strong", action="store_true", help="skip the strong-scaling (fixed-model) lines")
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed launches before each measurement's warmup (clock ramp)")
    ap.add_argument("--layout", default="slab", choices=["slab", "rows"],
                    help="HBM layout of the headline's peers: the PeerSlab tile-interleaved slab (default) or "
                         "one buffer per peer")
    ap.add_argument("--strong-steps", type=int, default=200,
                    help="timed steps of each strong-scaling line: the barrier that closes the timed region is "
                         "paid once per line, so short steps need many (an 8-way north-star bucket is ~19 us)")
    ap.add_argument("--leg-timeout", type=float, default=300.0,
                    help="seconds any one leg (the headline included) may take on any rank; past it the run "
                         "ends at once with a non-zero exit, rank 0 printing the line measured so far")
    ap.add_argument("--dist-timeout", type=float, default=0.0,
                    help="torch.distributed timeout in seconds (default: --leg-timeout + 120, so the leg "
                         "watchdog fires first)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch + rendezvous + rank-count check + bucket split + a gloo all-gather leg with its "
                         "parity check, no GPU work (what the CPU tests of the multi-rank launch run)")
    ap.add_argument("--sweep", action="store_true", help="interleaved A/B of launch variants, then exit")
    ap.add_argument("--host-breakdown", action="store_true", help="time the host-inclusive phases, then exit")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="do not restrict each rank's CPUs to its GPU's NUMA node (host_memory.bind_to_gpu_node)")
    ap.add_argument("--host-configs-only", action="store_true",
                    help="print the per-config host-inclusive table (CPU modules, real layouts), then exit")
    ap.add_argument("--device-configs-only", action="store_true",
                    help="print the device-resident module rounds (FedAvg.aggregate on HBM modules), then exit")
    ap.add_argument("--configs-only", action="store_true",
                    help="print the per-BASELINE-config device-resident table (no CPU legs), then exit")
    ap.add_argument("--sweep-cfgs", default="", help="variant,chunks,grid;... (default: built-in list)")
    ap.add_argument("--no-ceilings", action="store_true", help="skip the probe ceilings in --sweep")
    ap.add_argument("--libs", default="", help="comma list of libdlagg builds to A/B in --sweep (same process)")
    ap.add_argument("--pads", default="", help="comma list of extra row-pitch bytes to A/B in --sweep")
    ap.add_argument("--tile-bytes", default="", help="comma list of tile sizes: A/B the tile-interleaved slab "
                                                       "(dla_wsum_slab_tiled) against the row-major default in --sweep")
    return ap.parse_args()


def spawn_ranks(args) -> int:
    """``--gpus G`` without a torch.distributed.run wrapper: start G ranks (one process per
    GPU) through torch.distributed.run and return its exit code.  Runs before this process
    touches any GPU (no HIP call has been made yet), and starts the ranks as children."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, BENCH_SELF_SPAWNED="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // args.gpus)))
    return subprocess.call(cmd, env=env)


def args_cfg(args):
    return (args.variant, args.chunks, args.grid, args.block)


def setup_dist(args):
    """Returns (rank, world, device, cpu_group): cpu_group is a gloo group for host-side
    waits that must not park a kernel on any GPU (None at world 1).  Checks that the
    process group has exactly ``args.gpus`` ranks."""
    backend = args.dist_backend
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = None
    if not args.dry_run:
        dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
    cpu_group = None
    if world > 1:
        # every collective of the run has a deadline: no leg can wait out a 10-minute default
        # (the Legs watchdog, at --leg-timeout, ends a stuck run before this one fires)
        timeout = datetime.timedelta(seconds=args.dist_timeout or args.leg_timeout + 120)
        if backend == "nccl" and not args.dry_run:
            dist.init_process_group("nccl", device_id=dev, timeout=timeout)
        else:
            dist.init_process_group("gloo" if args.dry_run else backend, timeout=timeout)
        cpu_group = dist.new_group(backend="gloo", timeout=timeout)
        world = dist.get_world_size()
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the process group has %d rank(s)" % (args.gpus, world))
    return rank, world, dev, cpu_group


class LegAbort(Exception):
    """Some rank failed this leg before its collectives: every rank skips it."""


def _injected(leg, rank):
    """BENCH_INJECT_FAIL=<leg>:<rank>:<mode> (tests only): make `leg` fail on `rank` —
    raise_prepare (before its collectives), raise_run (right after every rank agreed to start
    them) or hang (block forever there)."""
    spec = os.environ.get("BENCH_INJECT_FAIL", "")
    if not spec:
        return None
    name, r, mode = spec.rsplit(":", 2)
    return mode if name == leg and int(r) == rank else None


class Legs:
    """Runs the legs of one bench process so that a failure or a hang on one rank never leaves the
    other ranks waiting in a collective:

    * a leg calls ``go()`` right before its first collective: a gloo all-reduce (MIN) of a ready
      flag.  A rank that failed while preparing contributes 0 there, and every rank skips the leg
      together (its row says "skipped");
    * a rank that fails AFTER ``go()`` (its peers may sit in a collective it will never join) ends
      the run at once with a non-zero exit, rank 0 printing the line measured so far
      ("aborted_leg"); ``settled()`` marks the end of a leg's collectives, after which a local
      failure is only recorded;
    * a watchdog thread ends the run the same way when a leg outlives ``timeout_s``;
    * after each leg the ranks agree (gloo, MIN) on its status and its parity flag, so a row's
      ``parity_ok`` is the verdict of every rank (None where no rank checked anything).
    At world 1 the agreements are no-ops and only the watchdog remains."""

    def __init__(self, rank, world, group, timeout_s, result):
        self.rank, self.world, self.group = rank, world, group
        self.timeout_s = timeout_s
        self.result = result  # the JSON line so far (printed by rank 0 if the run is cut short)
        self.failed = []
        self._name = None
        self._deadline = None
        self._went = self._go_done = False
        threading.Thread(target=self._watch, daemon=True).start()

    # ------------------------------------------------------------------ agreement / abort
    def _agree(self, vals):
        t = torch.tensor(vals, dtype=torch.int64)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return [int(x) for x in t]

    def go(self):
        """Every rank is ready for this leg's collectives (else LegAbort on every rank)."""
        if self._go_done:
            return
        self._go_done = True
        if not self._agree([1])[0]:
            raise LegAbort()
        self._went = True
        mode = _injected(self._name, self.rank)
        if mode == "raise_run":
            raise RuntimeError("injected failure after go() on rank %d" % self.rank)
        if mode == "hang":
            log("injected hang in leg %s on rank %d" % (self._name, self.rank), every_rank=True)
            while True:
                time.sleep(1)

    def settled(self):
        """This leg's collectives are over: a later local failure is recorded, not fatal."""
        self._went = False

    def fatal(self, leg, reason, code=1):
        log("FATAL in leg %s on rank %d: %s — ending the run" % (leg, self.rank, reason), every_rank=True)
        if self.rank == 0:
            for _ in range(3):
                try:
                    res = dict(self.result, aborted_leg={"leg": leg, "rank": 0, "reason": str(reason)[:500],
                                                         "exit_code": code})
                    print(json.dumps(res), flush=True)
                    break
                except (RuntimeError, TypeError, ValueError):  # the main thread was mutating the dict
                    time.sleep(0.05)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(code)

    def _watch(self):
        while True:
            time.sleep(0.25)
            d = self._deadline
            if d is not None and time.monotonic() > d:
                self.fatal(self._name, "leg exceeded its %.0f s deadline (--leg-timeout)" % self.timeout_s, 124)

    def arm(self, name, timeout_s=None):
        self._name = name
        self._deadline = time.monotonic() + (timeout_s or self.timeout_s)

    def disarm(self):
        self._deadline = None

    # ------------------------------------------------------------------ one leg
    def run(self, name, fn, *a, timeout_s=None, **kw):
        """Row of leg `name` (fn(self, *a, **kw) returns a dict; may set "parity_ok")."""
        self._went = self._go_done = False
        self.arm(name, timeout_s)
        log("leg %s" % name)
        row, ok = None, 1
        try:
            if _injected(name, self.rank) == "raise_prepare":
                raise RuntimeError("injected failure before the collectives on rank %d" % self.rank)
            row = fn(self, *a, **kw)
            if not self._go_done:
                self.go()
        except LegAbort:
            self.disarm()
            self.failed.append(name)
            return {"skipped": "a rank failed before this leg's collectives"}
        except Exception as exc:  # noqa: BLE001 — every failure of a leg is reported on its row
            if self._went:
                self.fatal(name, "%s: %s" % (type(exc).__name__, exc))
            msg = "%s: %s" % (type(exc).__name__, exc)
            log("leg %s failed on rank %d: %s" % (name, self.rank, msg), every_rank=True)
            if not self._go_done:  # the others are (or will be) in go(): tell them, skip together
                self._go_done = True
                try:
                    self._agree([0])
                except Exception as exc2:  # noqa: BLE001
                    self.fatal(name, "agreement failed: %s" % exc2)
                self.disarm()
                self.failed.append(name)
                return {"skipped": "failed on rank %d before its collectives" % self.rank, "error": msg}
            row, ok = {"error": msg}, 0
        par = row.get("parity_ok") if isinstance(row, dict) else None
        try:
            ok_all, par_all = self._agree([ok, 2 if par is None else int(bool(par))])
        except Exception as exc:  # noqa: BLE001 — a peer died: nothing can be agreed any more
            self.fatal(name, "final agreement failed: %s" % exc)
        self.disarm()
        if isinstance(row, dict):
            if par_all != 2:
                row["parity_ok"] = bool(par_all)
            if not ok_all and ok:
                row["error_on_another_rank"] = True
        if not ok_all or par_all == 0:
            self.failed.append(name)
        return row


def launch_info(world):
    return {"backend": dist.get_backend() if world > 1 else "none (single process)", "world_size": world,
            "started_by": ("bench.py --gpus (self-spawned torch.distributed.run)"
                           if os.environ.get("BENCH_SELF_SPAWNED") else
                           "torch.distributed.run" if "WORLD_SIZE" in os.environ else "single process")}


def log(msg, every_rank=False):
    """Progress on stderr (one line per phase), so a long run visibly advances."""
    rank = os.environ.get("RANK", "0")
    if rank == "0" or every_rank:
        print("[bench %.1fs r%s] %s" % (time.perf_counter() - _T0, rank, msg), file=sys.stderr, flush=True)


_T0 = time.perf_counter()


def barrier(world):
    if world > 1:
        dist.barrier()


def make_slab(n, p, dtype, device, seed_base):
    """Synthetic peers (BASELINE.md plan): per-peer seed, normal(0, 0.05)."""
    slab = torch.empty((n, p), dtype=dtype, device=device)
    for k in range(n):
        g = torch.Generator(device=device).manual_seed(seed_base + k)
        slab[k].normal_(0.0, 0.05, generator=g)
    return slab


class SlabInput:
    """n peers x p elements resident in HBM as PeerSlab holds them (core/peer_slab.py) and a
    prepared reduce of them into ``out``: layout "slab" = the tile-interleaved slab
    [n_tiles, n, tile] (fp32 / bf16 / f16; dla_wsum_slab_tiled), "rows" = one row per peer
    (separate peer buffers, what FedAvg.aggregate on device modules reduces; dla_wsum)."""

    def __init__(self, n, p, dt, device, seed_base, weights, layout="slab"):
        from accdfl_amd import _lib
        from accdfl_amd.core import wsum

        code = wsum.dtype_code(dt)
        pitch = max(128, (p + 127) // 128 * 128)
        rows = make_slab(n, pitch, dt, device, seed_base)
        self.out = torch.empty(pitch, dtype=dt, device=device)
        self.layout = layout if dt != torch.float64 else "rows"
        if self.layout == "slab":
            self.tile = _lib.slab_tile_elems(code, n, p)
            n_t = max(1, -(-p // self.tile))
            self.buf = torch.empty((n_t, n, self.tile), dtype=dt, device=device)
            full = p // self.tile
            for k in range(n):
                if full:
                    self.buf[:full, k, :].copy_(rows[k, : full * self.tile].view(full, self.tile))
                if p > full * self.tile:
                    self.buf[full, k, : p - full * self.tile].copy_(rows[k, full * self.tile: p])
            del rows
            self.plan = _lib.TiledPlan(code, self.buf.data_ptr(), self.tile, n, weights, p, self.out.data_ptr())
            self.kernel = "wsum_vec_kernel (tile-interleaved slab, %d-B tiles)" % (self.tile * self.buf.element_size())
        else:
            self.buf = rows
            self.tile = 0
            self.plan = _lib.Plan(code, [rows[k].data_ptr() for k in range(n)], weights, p, self.out.data_ptr())
            self.kernel = _lib.select_kernel(code, n, p)

    def launch(self, stream_ptr):
        self.plan.launch(stream_ptr)


SETTLE_S = 0.2  # --settle-ms: untimed launches before the warmup (GPU clocks ramp under load)


def time_kernel(fn, steps, warmup, world, settle_s=None):
    """Untimed launches for `settle_s` (the GPU ramps its clocks over the first tens of ms of
    load: a 25-launch run right after setup reads several % slow), `warmup` untimed calls,
    then exactly `steps` calls bracketed by barrier + synchronize; returns (wall seconds max
    over ranks, HIP-event seconds on the launch stream)."""
    settle_s = SETTLE_S if settle_s is None else settle_s
    if settle_s > 0:
        t_end = time.perf_counter() + settle_s
        while time.perf_counter() < t_end:
            for _ in range(8):
                fn()
            torch.cuda.synchronize()
    for _ in range(warmup):
        fn()
    stream = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev_s = ev0.elapsed_time(ev1) / 1e3
    if world > 1:
        on_gpu = dist.get_backend() == "nccl"
        t = torch.tensor([wall, ev_s], dtype=torch.float64, device="cuda" if on_gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, ev_s = float(t[0]), float(t[1])
    return wall, ev_s


def cpu_threads():
    """(threads used for the CPU legs, how that count was found).  The process's CPU
    affinity is what it may run on; on the GPU box the job's share is
    also set as OMP_NUM_THREADS (the affinity there can list the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if omp and omp < aff:
        return omp, "OMP_NUM_THREADS=%d (the job's CPU share; sched_getaffinity lists %d)" % (omp, aff)
    return aff, "len(os.sched_getaffinity(0)) = %d" % aff


def _cgroup_cpus():
    """CPUs the cgroup quota allows (cpu.max), or None when unlimited / unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


_COLD_SCRIPT = r"""
import json, statistics, sys, time
import numpy as np, torch
sys.path.insert(0, sys.argv[1])
from oracle.fedavg_oracle import fedavg_flat_torch
n, p, th, budget = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5])
torch.set_num_threads(th)
gen = torch.Generator().manual_seed(1000)
peers = [torch.randn(p, generator=gen) * 0.05 for _ in range(n)]
w = [float(x) for x in np.random.default_rng(0).dirichlet(np.ones(n))]
out = torch.empty(p)
fedavg_flat_torch(peers, w, out)
ts, start = [], time.perf_counter()
while (time.perf_counter() - start < budget and len(ts) < 50) or len(ts) < 2:
    t0 = time.perf_counter()
    fedavg_flat_torch(peers, w, out)
    ts.append(time.perf_counter() - t0)
print(json.dumps({"median_ms": statistics.median(ts) * 1e3, "reduces": len(ts)}))
"""


def cpu_baseline_cold(n, p, threads, budget_s):
    """The literal reference op sequence (a fresh ``w * p`` temporary per peer) in a FRESH
    process: what a newly started reference process pays, page faults of every temporary
    included (the in-process figure depends on what the allocator already holds)."""
    try:
        r = subprocess.run([sys.executable, "-c", _COLD_SCRIPT, ROOT, str(n), str(p), str(threads), str(budget_s)],
                           capture_output=True, text=True, timeout=120 + 4 * budget_s,
                           env=dict(os.environ, OMP_NUM_THREADS=str(threads)))
        row = json.loads(r.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError) as exc:
        return {"error": "%s: %s" % (type(exc).__name__, exc)}
    return {"GB/s": round((n + 1) * p * 4 / (row["median_ms"] / 1e3) / 1e9, 3),
            "median_ms": round(row["median_ms"], 1), "reduces": row["reduces"], "threads": threads}


def cpu_baseline(n, p, budget_s, headline=None):
    """The reference op sequence (deepcopy -> mul_(0) -> add_(w*p)) on torch-CPU, timed on a
    bounded sample of the same workload: repeated full NS reduces until ~budget_s, at the
    process's CPU share (cpu_threads), at every affinity CPU when that differs, and on one
    thread, with the product temporary in a held buffer (fedavg_flat_torch_warm: same ops,
    same bits, no page faults — the sequence at its best).  ``value`` / ``cores`` is the
    fastest of these counts.  ``cold_fresh_process`` times the literal sequence (a fresh
    temporary per peer) in a new process at the same thread count.

    ``headline``: (the headline's own peers copied to host, its output copied to host).  The timed
    reduces then run on exactly the headline's inputs, and the output of the last one is compared
    bit for bit, every element, with the output the timed GPU headline produced
    (``headline_oracle_parity``): the driver's bench line is checked against the reference's
    arithmetic in the run that produced it."""
    sys.path.insert(0, ROOT)
    from oracle.fedavg_oracle import fedavg_flat_torch_warm  # timed CPU baseline (kind "port")

    share, how = cpu_threads()
    aff = len(os.sched_getaffinity(0))
    if headline is not None:
        peers, head_out = headline
    else:
        gen = torch.Generator().manual_seed(1000)
        peers = [torch.randn(p, generator=gen) * 0.05 for _ in range(n)]
        head_out = None
    w = [float(x) for x in np.random.default_rng(0).dirichlet(np.ones(n))]
    out = torch.empty(p)
    tmp = torch.empty(p)
    byts = (n + 1) * p * 4
    quota = _cgroup_cpus()
    # every affinity CPU as well, unless the cgroup quota caps the job below that count (then
    # oversubscribed threads only measure throttling: 2.4 s vs 0.15 s per reduce at 256 threads
    # under a 16-CPU quota, profiles/r02a_bench.log)
    counts = [share] + ([aff] if aff != share and (quota is None or quota >= aff) else []) + [1]
    per = {}
    for th in counts:
        torch.set_num_threads(th)
        fedavg_flat_torch_warm(peers, w, out, tmp)  # warm-up
        times = []
        start = time.perf_counter()
        lim = budget_s if th != 1 else budget_s / 2
        while (time.perf_counter() - start < lim and len(times) < 200) or len(times) < 2:
            t0 = time.perf_counter()
            fedavg_flat_torch_warm(peers, w, out, tmp)
            times.append(time.perf_counter() - t0)
        med = statistics.median(times)
        per[th] = (med, len(times), sum(times))
        log("cpu baseline: %d threads, %.1f ms per reduce" % (th, med * 1e3))
    torch.set_num_threads(share)
    best = min((v[0], th) for th, v in per.items())[1]
    med, cnt, tot = per[best]
    check = None
    if head_out is not None:
        same = torch.equal(out.view(torch.int32), head_out.view(torch.int32))
        bad = 0 if same else int((out.view(torch.int32) != head_out.view(torch.int32)).sum())
        check = {"parity_ok": bool(same), "elements": p, "mismatches": bad,
                 "check": "the timed GPU headline's output (every element, D2H after the timed region) == the "
                          "reference op sequence (oracle port, fedavg.py:20-25) on the same %d peers, bit for bit" % n}
        log("cpu baseline: headline vs oracle port on the same peers: %s" % ("bit-exact" if same else
                                                                           "%d mismatches" % bad))
    del peers, out, tmp, head_out
    log("cpu baseline: literal op sequence in a fresh process")
    cold = cpu_baseline_cold(n, p, share, min(4.0, budget_s))
    return {
        "value": round(byts / med / 1e9, 3),
        "unit": "GB/s",
        "cores": best,
        "kind": "port",
        "sample": "%d full reduces of %d peers x %d fp32 (torch-CPU op sequence of fedavg.py:20-25, product "
                  "temporary held) on %d threads, median %.1f ms, %.1f s total" % (cnt, n, p, best, med * 1e3, tot),
        "threads_source": how,
        "affinity_cpus": aff,
        "cgroup_cpu_quota": quota,
        "by_threads": {str(th): {"GB/s": round(byts / v[0] / 1e9, 3), "median_ms": round(v[0] * 1e3, 1),
                                 "reduces": v[1]} for th, v in per.items()},
        "value_1thread": round(byts / per[1][0] / 1e9, 3),
        "regime": ("LLC-assisted: the held product temporary and the running sum (2 x %d MiB) stay in the "
                   "CPU's last-level cache across peers, so only the peer reads come from DRAM; not a DRAM "
                   "rate. cold_fresh_process is the literal sequence, page faults included" % (p * 4 >> 20)),
        "cold_fresh_process": cold,
        "cpu": _cpu_model(),
        "headline_oracle_parity": check,
        "sample_inputs": "the headline's own peers (copied from HBM)" if check is not None else
                         "seeded CPU peers (torch.Generator 1000)",
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def host_inclusive(n, p, reps=5):
    """FedAvg.aggregate on CPU modules (the reference call sites) end to end."""
    from torch import nn

    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    gen = torch.Generator().manual_seed(2000)
    models = []
    for _ in range(n):
        m = nn.Module()
        m.w = nn.Parameter(torch.randn(p, generator=gen) * 0.05)
        models.append(m)
    w = [float(1.0 / n)] * n
    FedAvg.aggregate(models, w)
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        FedAvg.aggregate(models, w)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"value": round((n + 1) * p * 4 / med / 1e9, 3), "unit": "GB/s", "ms": round(med * 1e3, 2),
            "path": "FedAvg.aggregate(CPU nn.Modules): deepcopy (params uninitialised, pooled pageable) + "
                    "dla_host_reduce (threaded pack of each 32 MiB chunk into page-locked rows, one H2D DMA per "
                    "chunk, reduce, D2H and unpack into the result, two chunks in flight)"}


def host_inclusive_sharded(n, p, n_devices, reps=3):
    """SURVEY.md §8(e) host-inclusive scaling line: FedAvg.aggregate on CPU modules (the
    reference call sites) with the flat model bucket-sharded over GPUs 0..n_devices-1 of
    THIS process, each bucket crossing its own GPU's PCIe link.  The same model at every
    device count (strong scaling); the result is bit-identical for any count."""
    from torch import nn

    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    gen = torch.Generator().manual_seed(2000)
    models = []
    for _ in range(n):
        m = nn.Module()
        m.w = nn.Parameter(torch.randn(p, generator=gen) * 0.05)
        models.append(m)
    w = [float(x) for x in np.random.default_rng(3).dirichlet(np.ones(n))]
    res = {}
    # one visible GPU (the several-ranks rehearsal): the buckets repeat GPU 0, the same code path
    devices = list(range(n_devices)) if n_devices <= torch.cuda.device_count() else [0] * n_devices
    runs = [([0], True)] + ([(devices, True), (devices, False)] if n_devices > 1 else [])
    ref = None
    ok = True
    for devs, threads in runs:
        fa.set_host_devices(devs)
        fa.set_shard_threads(threads)
        try:
            out = fa.FedAvg.aggregate(models, w)
            if ref is None:
                ref = out.w.detach().clone()  # the one-GPU result: every sharded result must equal it
            good = same_bits(out.w.detach(), ref)
            ok = ok and good
            del out
            times = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fa.FedAvg.aggregate(models, w)
                times.append(time.perf_counter() - t0)
        finally:
            fa.set_host_devices([])
            fa.set_shard_threads(True)
            fa.release_staging()
        med = statistics.median(times)
        key = "%d_gpu" % len(devs) + ("" if len(devs) == 1 else ("_native" if threads else "_packed"))
        res[key] = {"ms": round(med * 1e3, 2), "GB/s": round((n + 1) * p * 4 / med / 1e9, 2), "devices": devs,
                    "parity_ok": good}
    res["path"] = ("FedAvg.aggregate(CPU nn.Modules), %d x %d fp32, bucket-sharded over the GPUs of one "
                   "process (fedavg.set_host_devices); each sharded result checked bit for bit against the "
                   "one-GPU result" % (n, p))
    res["parity_ok"] = ok
    return res


def host_breakdown(n, p, device):
    """Phases of FedAvg.aggregate on CPU modules (the host-inclusive path), timed apart."""
    import copy

    from torch import nn

    gen = torch.Generator().manual_seed(2000)
    models = []
    for _ in range(n):
        m = nn.Module()
        m.w = nn.Parameter(torch.randn(p, generator=gen) * 0.05)
        models.append(m)
    pinned = torch.empty((n, p), pin_memory=True)
    dev = torch.empty((n, p), device=device)
    out = torch.empty(p, device=device)
    h_out = torch.empty(p, pin_memory=True)
    res = {}

    def t(name, fn, reps=3):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res[name] = round(min(ts) * 1e3, 2)

    t("deepcopy_model0_ms", lambda: copy.deepcopy(models[0]))
    t("pack_pinned_ms", lambda: [pinned[k].copy_(models[k].w.detach()) for k in range(n)])
    t("h2d_pinned_ms", lambda: dev.copy_(pinned, non_blocking=True))
    t("h2d_pageable_ms", lambda: [dev[k].copy_(models[k].w.detach(), non_blocking=False) for k in range(n)])
    from accdfl_amd.core import wsum
    t("reduce_ms", lambda: wsum.wsum_rows(dev, [1.0 / n] * n, p, out=out))
    t("d2h_pinned_ms", lambda: h_out.copy_(out, non_blocking=True))
    c = copy.deepcopy(models[0])
    t("unpack_ms", lambda: c.w.data.copy_(h_out))
    # f1 wire ingress of one peer (serialize_model bytes of a 25 M fp32 model)
    import pickle

    from accdfl_amd.core import wire
    from accdfl_amd.core.peer_slab import PeerSlab

    data = wire.serialize_model(models[0])
    res["wire_payload_MB"] = round(len(data) / 1e6, 1)
    t("wire_safe_decode_ms", lambda: wire.loads_state_dict(data, copy=False))
    t("reference_decode_pickle_loads_ms", lambda: pickle.loads(data))  # our own bytes
    sd = wire.loads_state_dict(data)
    t("reference_load_state_dict_ms", lambda: c.load_state_dict(sd))
    slab = PeerSlab([(p,)], torch.float32, capacity=1, device=device)

    def stage():
        slab.reset()
        slab.stage([sd["w"]])
        slab.copy_stream.synchronize()
    t("wire_stage_h2d_ms", stage)
    res["threads"] = torch.get_num_threads()
    return res


def _comm_device(device):
    """Where the collectives' tensors live: the GPU over RCCL, the host over gloo (the
    several-ranks-on-one-GPU rehearsal)."""
    return device if dist.get_backend() == "nccl" else torch.device("cpu")


def _bits(t):
    return t.view({8: torch.int64, 4: torch.int32, 2: torch.int16}[t.element_size()])


def same_bits(a, b):
    """Bit-for-bit equality of two float tensors (NaN-free synthetic data), on a's device."""
    a = a.contiguous()
    b = b.to(a.device).contiguous()
    return a.shape == b.shape and a.dtype == b.dtype and bool(torch.equal(_bits(a), _bits(b)))


def gather_all(local, max_len, cdev):
    """all_gather of `local` (padded to max_len elements) -> one tensor per rank, on every rank."""
    buf = torch.zeros(max_len, dtype=local.dtype, device=cdev)
    if local.numel():
        buf[: local.numel()].copy_(local)
    outs = [torch.empty_like(buf) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, buf)
    return outs


def _seeded_rows(ks, length, dt, device, seed_base):
    """Rows k in ks of a seeded peer set (row k = normal(0, 0.05) of `length` elements from
    seed seed_base + k): every rank and the rank-0 reference build the same rows."""
    out = torch.empty((len(ks), length), dtype=dt, device=device)
    for i, k in enumerate(ks):
        out[i].normal_(0.0, 0.05, generator=torch.Generator(device=device).manual_seed(seed_base + k))
    return out


def _rank_content(r, length, dt, cdev):
    """A rank's deterministic all-gather payload (cheap to rebuild on every rank)."""
    i = torch.arange(length, dtype=torch.int64, device=cdev)
    return ((i * 7 + r * 1_000_003) % 65521).to(dt)


def leg_headline_parity(legs, inp, n, p, dt, w, rank, world, device):
    """The weak headline's per-rank buckets, reassembled by an all-gather, against ONE single-GPU
    reduce of the whole n x (world * p) model rebuilt on rank 0 from the same seeds (rank r's
    bucket of peer k = seed 1000 + 97 r + k) — bit for bit."""
    from accdfl_amd.core import wsum

    cdev = _comm_device(device)
    ref = None
    if rank == 0:
        pitch = max(128, (p + 127) // 128 * 128)
        full = torch.empty((n, world * p), dtype=dt, device=device)
        for r in range(world):
            full[:, r * p:(r + 1) * p].copy_(make_slab(n, pitch, dt, device, 1000 + 97 * r)[:, :p])
        ref = wsum.wsum(list(full), w)
        del full
    legs.go()
    got = gather_all(inp.out[:p], p, cdev)
    legs.settled()
    row = {"check": "all-gathered buckets of every rank == one reduce of the whole %d x %d model on rank 0's GPU"
                    % (n, world * p)}
    if rank == 0:
        row["parity_ok"] = same_bits(torch.cat(got).to(device), ref)
    return row


def leg_allgather(legs, p, dt, es, world, rank, device, iters=10):
    """RCCL all-gather of every rank's averaged bucket into the whole model on every rank (the
    reassembly step, never inside `value`); every rank checks the gathered model against the
    buckets it can rebuild (_rank_content)."""
    from accdfl_amd.core.sharding import BucketShardedFedAvg

    cdev = _comm_device(device)
    sh = BucketShardedFedAvg(p * world, dt, device=cdev)
    bucket = _rank_content(rank, sh.bucket_len, dt, cdev)
    full = torch.empty(p * world, dtype=dt, device=cdev)
    want = torch.cat([_rank_content(r, sh.bucket_len, dt, cdev) for r in range(world)])[: p * world]
    legs.go()
    wall, _ = time_kernel(lambda: sh.all_gather(bucket, full), iters, 2, world, settle_s=0)
    legs.settled()
    return {"ms": round(wall / iters * 1e3, 3), "bytes_out_per_rank": p * world * es,
            "GBps_per_rank_in": round((world - 1) * sh.bucket_len * es / (wall / iters) / 1e9, 1),
            "parity_ok": same_bits(full, want)}


def leg_peer_sharded(legs, exact, n, p, dt, world, rank, device, w, iters=10):
    """Peers arriving whole on different ranks (rank r holds peers r*m .. r*m+m-1, m = n / world,
    each of world * p elements, seed 6000 + k):
    * exact: all-to-all transpose -> the same list-order bucket reduce -> all-gather, checked bit
      for bit against one single-GPU reduce of all n peers on rank 0;
    * reduce-scatter (exact=False): local partial fold -> reduce-scatter -> all-gather, checked
      against the same reference within its stated bound |err| <= N 2^-23 sum_k |w_k p_k|."""
    from accdfl_amd.core import wsum
    from accdfl_amd.core.sharding import BucketShardedFedAvg

    if n % world:
        return {"skipped": "%d peers do not split evenly over %d ranks" % (n, world)}
    if not exact and dt not in (torch.float32, torch.float64):
        return {"skipped": "the reduce-scatter mode states its bound for fp32 / fp64 only"}
    cdev = _comm_device(device)
    on_gpu = cdev.type == "cuda"
    m = n // world
    L = p * world

    def reducer(peers, weights, out):
        if on_gpu:
            return wsum.wsum(list(peers), weights, out=out)
        out.copy_(wsum.wsum([t.to(device) for t in peers], weights).cpu())
        return out

    local = _seeded_rows(range(rank * m, (rank + 1) * m), L, dt, device, 6000).to(cdev)
    ref = bound = None
    if rank == 0:
        allp = _seeded_rows(range(n), L, dt, device, 6000)
        ref = wsum.wsum(list(allp), w)
        if not exact:
            bound = torch.zeros(L, dtype=torch.float64, device=device)
            for k in range(n):
                bound.add_(allp[k].double().abs_().mul_(abs(w[k])))
            bound.mul_(n * 2.0 ** -23)
        del allp
    sh = BucketShardedFedAvg(L, dt, device=cdev, reducer=reducer)
    fn = lambda: sh.aggregate_peer_sharded(local, w, exact=exact)  # noqa: E731
    legs.go()
    wall, _ = time_kernel(fn, iters, 2, world, settle_s=0)
    out = fn()
    legs.settled()
    row = {"ms": round(wall / iters * 1e3, 3), "peers_per_rank": m, "model_params": L, "bit_exact": exact}
    if rank == 0:
        got = out.to(device)
        if exact:
            row["parity_ok"] = same_bits(got, ref)
        else:
            err = (got.double() - ref.double()).abs_()
            row["parity_ok"] = bool(torch.all(err <= bound))
            row["max_err_over_bound"] = float((err / bound.clamp_min(1e-300)).max())
            row["tolerance"] = "N * 2^-23 * sum_k |w_k p_k| (DESIGN.md §2)"
    return row


def leg_xgmi_sharded(legs, n, p, world, rank, device, w, reps=10):
    """dla_wsum_sharded (ONE process, several GPUs): n peers of p fp32 placed
    round-robin on GPUs 0..G-1 of rank 0's process, G = min(world, visible GPUs); shard s reduces
    bucket s of every peer on GPU s, reading the peers held elsewhere over xGMI; "direct" writes
    every bucket straight into the result on GPU 0, "gather" writes locally then copies
    peer-to-peer.  Checked bit for bit against wsum on GPU 0.  With one visible GPU (the
    several-ranks rehearsal) the shards repeat GPU 0.  The other ranks idle on the CPU."""
    from accdfl_amd.core import wsum

    legs.go()
    if rank != 0:
        return {}
    g = min(world, torch.cuda.device_count())
    devs = [torch.device("cuda", i) for i in range(g)] if g > 1 else [torch.device("cuda", 0)] * world
    uniq = sorted({d.index for d in devs})
    pitch = max(128, (p + 127) // 128 * 128)
    rows = make_slab(n, pitch, torch.float32, device, 7000)
    ref = wsum.wsum([rows[k, :p] for k in range(n)], w)
    peers = [rows[k, :p].to(devs[k % len(devs)]) for k in range(n)]
    torch.cuda.synchronize()

    def sync():
        for d in uniq:
            torch.cuda.synchronize(d)

    row = {"devices": [d.index for d in devs], "peer_devices": [t.device.index for t in peers],
           "peers": n, "params": p, "modes": {}}
    ok = True
    for mode in ("direct", "gather"):
        out = wsum.wsum_sharded(peers, w, devs, mode=mode)
        sync()
        good = same_bits(out, ref)
        ok = ok and good
        t0 = time.perf_counter()
        for _ in range(reps):
            wsum.wsum_sharded(peers, w, devs, out=out, mode=mode)
        sync()
        t = (time.perf_counter() - t0) / reps
        row["modes"][mode] = {"ms": round(t * 1e3, 3), "GB/s": round((n + 1) * p * 4 / t / 1e9, 1),
                              "parity_ok": good}
    row["parity_ok"] = ok
    return row


GNLENET = [(32, 3, 5, 5), (32,), (32,), (32,), (32, 32, 5, 5), (32,), (32,), (32,), (64, 32, 5, 5), (64,),
           (64,), (64,), (10, 576), (10,)]  # accdfl/core/models/cifar10.py GNLeNet parameters


def _gnlenet_models(n, layers=False):
    """n GNLeNet-layout CPU models: one ParameterList of the 14 tensors, or (layers) the module tree of
    layers the reference's model class builds (conv / pool / GroupNorm / linear submodules,
    accdfl/core/models/cifar10.py) with the same parameters in the same order — the result's deepcopy
    then clones nine modules with their hook dicts and attributes, as at the reference's call sites."""
    from torch import nn

    g = torch.Generator().manual_seed(n)
    if not layers:
        return [nn.ParameterList([nn.Parameter(torch.randn(s, generator=g) * 0.05) for s in GNLENET])
                for _ in range(n)]
    out = []
    for _ in range(n):
        m = nn.Module()
        m.conv1 = nn.Conv2d(3, 32, 5, padding="same")
        m.pool = nn.MaxPool2d(2, 2)
        m.gn1 = nn.GroupNorm(2, 32)
        m.conv2 = nn.Conv2d(32, 32, 5, padding="same")
        m.gn2 = nn.GroupNorm(2, 32)
        m.conv3 = nn.Conv2d(32, 64, 5, padding="same")
        m.gn3 = nn.GroupNorm(2, 64)
        m.fc1 = nn.Linear(576, 10)
        with torch.no_grad():
            for p, s in zip(m.parameters(), GNLENET):
                assert tuple(p.shape) == s
                p.copy_(torch.randn(s, generator=g) * 0.05)
        out.append(m)
    return out


def _median_ms(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e3, 3)


LAYOUTS_FILE = os.path.join(ROOT, "tests", "golden", "layouts.json")  # recorded from the reference's create_model

# (layout, peers, dtype) of every GPU config's WHOLE model as the reference aggregator holds it:
# N CPU modules with the real parameter / buffer layout (SURVEY.md §8d host-inclusive rate).
HOST_CONFIGS = {
    "configs[1] CIFAR-10 GNLeNet, 8 peers": ("gnlenet", 8, "f32"),
    "configs[2] FEMNIST CNN, 32 peers": ("femnist_cnn", 32, "f32"),
    "configs[3] CIFAR-10 GNLeNet, 64 peers": ("gnlenet", 64, "f32"),
    "configs[3'] CIFAR-10 ResNet-8, 64 peers": ("cifar10_resnet8", 64, "f32"),
    "configs[4] google_speech ResNet-34, 128 peers, bf16": ("google_speech_resnet34", 128, "bf16"),
}


def _layout(name):
    if name == "gnlenet":
        return [list(s) for s in GNLENET], []
    lay = json.load(open(LAYOUTS_FILE))[name]
    return [s for _, s, _ in lay["params"]], [(s, d) for _, s, d in lay["buffers"]]


def _layout_models(name, n, dt, pinned, seed=4000):
    """n CPU modules with the layout `name`: one tensor per parameter (pageable, allocated
    apart as load_state_dict leaves them) or views of one page-locked row per peer (what a
    page-locked ingress buffer holds, e.g. DeviceModelManager's EVA gather); BN buffers as
    the reference models carry them.  Values: one seeded normal(0, 0.05) base scaled per
    peer (the values do not change any timing)."""
    from torch import nn

    shapes, bufs = _layout(name)
    numels = [int(np.prod(s)) if s else 1 for s in shapes]
    base = torch.randn(sum(numels), generator=torch.Generator().manual_seed(seed)) * 0.05
    models = []
    for k in range(n):
        flat = (base * (1.0 + 0.001 * k)).to(dt)
        if pinned:
            flat = flat.pin_memory()
            parts = [t.view(s) for t, s in zip(flat.split(numels), shapes)]
        else:
            parts = [t.view(s).clone() for t, s in zip(flat.split(numels), shapes)]
        m = nn.Module()
        m.ps = nn.ParameterList([nn.Parameter(t) for t in parts])
        for j, (s, bdt) in enumerate(bufs):
            m.register_buffer("b%d" % j, torch.zeros(s, dtype=getattr(torch, bdt)))
        models.append(m)
        del flat
    return models, sum(numels)


def host_inclusive_configs(reps=3):
    """FedAvg.aggregate on every GPU config's whole model as CPU modules with the reference's
    real layout, end to end (deepcopy, H2D of N x P, reduce, D2H into the result), with the
    peers' parameters pageable (every reference call site) and page-locked (peers decoded into
    page-locked ingress buffers).  The reference op sequence on the same pageable modules is
    timed in the cpu_baseline leg (cpu_layout_configs)."""
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg, release_staging

    res = {}
    for name, (lay, n, dts) in HOST_CONFIGS.items():
        dt = torch.float32 if dts == "f32" else torch.bfloat16
        es = 4 if dts == "f32" else 2
        row = {"peers": n, "dtype": dts}
        for mem in ("pageable", "pinned"):
            log("host-inclusive %s (%s peers)" % (name, mem))
            models, p = _layout_models(lay, n, dt, mem == "pinned")
            w = [float(1.0 / n)] * n
            ms = _median_ms(lambda: FedAvg.aggregate(models, w), reps)
            row["params"] = p
            row["tensors"] = len(list(models[0].parameters()))
            row[mem + "_ms"] = ms
            row[mem + "_GB/s"] = round((n + 1) * p * es / (ms / 1e3) / 1e9, 2)
            if mem == "pageable":
                log("host-inclusive %s (staged on arrival)" % name)
                row.update(staged_on_arrival(models, w))
            del models
        row["h2d_bytes"] = n * p * es
        res[name] = row
    release_staging()
    return res


def staged_on_arrival(models, w, reps=3):
    """The same CPU modules handed to DeviceModelManager one by one as they would arrive
    (accdfl/core/model_manager.py:42-47 process_incoming_trained_model; the GL / DL call sites,
    accdfl/gl/community.py:110-117, accdfl/dl/community.py:98-106): each is staged into the HBM PeerSlab
    on arrival, and the next arrives only after its copy has finished (a gap at least as long as each
    H2D).  ``staged_on_arrival_ms``: from the LAST arrival (its process_incoming_trained_model call) to
    aggregate_trained_models returning the CPU result module — the last model's H2D, the reduce, the
    D2H into the result and deepcopy(models[0]).  ``staged_parity_ok``: the result equals FedAvg.aggregate
    of the same modules (the host path), every parameter bit for bit."""
    from types import SimpleNamespace

    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg
    from accdfl_amd.core.model_manager import DeviceModelManager

    n = len(models)
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0,
                            capacity=n)
    ts, out = [], None
    for _ in range(reps + 1):
        mm.reset_incoming_trained_models()
        for k, m in enumerate(models[:-1]):
            mm.process_incoming_trained_model(b"p%d" % k, m)
            mm.slab.copy_stream.synchronize()  # the next model arrives after this one's H2D
        time.sleep(0.002)
        t0 = time.perf_counter()
        mm.process_incoming_trained_model(b"last", models[-1])
        out = mm.aggregate_trained_models(w)
        ts.append(time.perf_counter() - t0)
    uniform = mm._uniform()
    want = FedAvg.aggregate(models, w)
    ok = all(torch.equal(a.detach().view(-1).view(torch.uint8), b.detach().view(-1).view(torch.uint8))
             for a, b in zip(out.parameters(), want.parameters()))
    del mm
    torch.cuda.empty_cache()
    return {"staged_on_arrival_ms": round(statistics.median(ts[1:]) * 1e3, 3), "staged_slab_path": uniform,
            "staged_parity_ok": bool(ok)}


# (layout, peers, dtype) of the device-resident module rounds: FedAvg.aggregate on modules that live in
# HBM (models trained on the GPU; the simulators' averages), the reference layouts at their peer counts
DEVICE_CONFIGS = {
    "configs[1] CIFAR-10 GNLeNet, 8 peers": ("gnlenet", 8, "f32"),
    "configs[2] FEMNIST CNN, 32 peers": ("femnist_cnn", 32, "f32"),
    "configs[3] CIFAR-10 GNLeNet, 64 peers (whole model)": ("gnlenet", 64, "f32"),
    "configs[3'] CIFAR-10 ResNet-8, 64 peers (whole model)": ("cifar10_resnet8", 64, "f32"),
    "configs[4] google_speech ResNet-34, 16 peers, bf16": ("google_speech_resnet34", 16, "bf16"),
    "configs[4] google_speech ResNet-34, 128 peers, bf16 (whole model)": ("google_speech_resnet34", 128, "bf16"),
}


def _device_layout_models(name, n, dt, device, seed=4100):
    """n device-resident modules with the layout `name` (one tensor per parameter, allocated apart
    as .to(device) of a trained model leaves them), BN buffers as the reference models carry them."""
    from torch import nn

    shapes, bufs = _layout(name)
    numels = [int(np.prod(s)) if s else 1 for s in shapes]
    base = torch.randn(sum(numels), generator=torch.Generator().manual_seed(seed)).to(device) * 0.05
    models = []
    for k in range(n):
        flat = (base * (1.0 + 0.001 * k)).to(dt)
        m = nn.Module()
        m.ps = nn.ParameterList([nn.Parameter(t.view(s).clone()) for t, s in zip(flat.split(numels), shapes)])
        for j, (s, bdt) in enumerate(bufs):
            m.register_buffer("b%d" % j, torch.zeros(s, dtype=getattr(torch, bdt), device=device))
        models.append(m)
        del flat
    return models, sum(numels)


def device_module_configs(device, reps=10):
    """FedAvg.aggregate on DEVICE-resident modules of the reference layouts (the
    reference walks every parameter of every model, fedavg.py:24; the simulators average many
    models, simulations/gl/gl_simulation.py:96-105), beside the flat PeerSlab reduce of the same
    bytes.  Per config:
      * end_to_end_ms: the whole FedAvg.aggregate call (parameter walk, deepcopy of models[0], pointer
        table, reduce) until the result is ready (synchronised);
      * layout_walk_ms: of which the one-pass walk over every parameter of every model
        (fedavg._device_layout: shapes, dtype, device, contiguity, pointers);
      * reduce_us: the device reduce alone, back to back on the walked layout (HIP events over the
        timed region): the table's H2D copy + one wsum_multi_vec_kernel launch per 128-peer pass;
      * per_tensor_reduce_us: the same reduce through the round-2 path (dla_wsum_multi: tensors packed
        32 per launch up to 32 peers, one launch per tensor above);
      * flat_slab_us: the tile-interleaved PeerSlab reduce of the same (N + 1) x P x s bytes
        (what DeviceModelManager reduces), HIP events over a prepared launch."""
    import ctypes

    from accdfl_amd.core import wsum
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    res = {}
    for name, (lay, n, dts) in DEVICE_CONFIGS.items():
        log("device modules: " + name)
        dt = torch.float32 if dts == "f32" else torch.bfloat16
        es = 4 if dts == "f32" else 2
        models, p = _device_layout_models(lay, n, dt, device)
        w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]
        byts = (n + 1) * p * es

        def e2e():
            fa.FedAvg.aggregate(models, w)
            torch.cuda.synchronize()

        row = {"peers": n, "params": p, "dtype": dts, "tensors": len(list(models[0].parameters())),
               "bytes": byts, "end_to_end_ms": _median_ms(e2e, reps),
               "layout_walk_ms": _median_ms(lambda: fa._device_layout(models), reps)}
        dtype_, dev_, numels, table = fa._device_layout(models)
        center = fa._center_copy(models[0])
        outs = (ctypes.c_void_p * len(numels))(*[c.data_ptr() for c in center.parameters()])
        nums = (ctypes.c_int64 * len(numels))(*numels)
        ptrs = (ctypes.c_void_p * table.size).from_buffer(table)
        steps = 20 if byts > (256 << 20) else 100

        def reduce_once():
            wsum.wsum_multi_ptrs(dt, ptrs, outs, nums, w, device)

        ev = statistics.median(time_kernel(reduce_once, steps, 5, 1, settle_s=0.05)[1] for _ in range(3))
        row["reduce_us"] = round(ev / steps * 1e6, 2)
        row["reduce_GB/s"] = round(byts / (ev / steps) / 1e9, 1)
        old = wsum.MULTI_TABLE_MIN_PEERS, wsum.MULTI_TABLE_MIN_BYTES
        wsum.MULTI_TABLE_MIN_PEERS = wsum.MULTI_TABLE_MIN_BYTES = 1 << 62
        try:
            ev = statistics.median(time_kernel(reduce_once, steps, 5, 1, settle_s=0.05)[1] for _ in range(3))
        finally:
            wsum.MULTI_TABLE_MIN_PEERS, wsum.MULTI_TABLE_MIN_BYTES = old
        row["per_tensor_reduce_us"] = round(ev / steps * 1e6, 2)
        del models, center
        torch.cuda.empty_cache()
        inp = SlabInput(n, p, dt, device, 1000, w)
        sp = torch.cuda.current_stream().cuda_stream
        ev = statistics.median(time_kernel(lambda: inp.launch(sp), steps, 5, 1, settle_s=0.05)[1] for _ in range(3))
        row["flat_slab_us"] = round(ev / steps * 1e6, 2)
        row["reduce_over_flat_slab"] = round(row["reduce_us"] / row["flat_slab_us"], 3)
        row["regime"] = "HBM" if byts > (256 << 20) else "Infinity-Cache / launch-latency"
        del inp
        torch.cuda.empty_cache()
        res[name] = row
    res[TREE_CONFIG] = device_tree_round(device, reps)
    return res


# the simulators' device models are the reference's module trees, not one ParameterList per model
TREE_CONFIG = "configs[4] google_speech ResNet-34, 16 peers, bf16 (reference module tree)"


def device_tree_round(device, reps=10):
    """FedAvg.aggregate on 16 device-resident google_speech ResNet-34 models built as the reference's
    module tree (97 modules; tests/test_center_copy_layouts.py tree_from_layout, from the layouts the
    reference's create_model gives), holding the same values as the ParameterList models of
    device_module_configs: end to end and the layout walk, and ``parity_ok`` — the tree round's result
    equals the ParameterList round's, every parameter bit for bit."""
    from accdfl_amd.core.gradient_aggregation import fedavg as fa

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_center_copy_layouts import tree_from_layout

    log("device modules: " + TREE_CONFIG)
    flat, p = _device_layout_models("google_speech_resnet34", 16, torch.bfloat16, device)
    trees = []
    for fm in flat:
        t = tree_from_layout("google_speech_resnet34").to(device=device, dtype=torch.bfloat16)
        with torch.no_grad():
            for q, src in zip(t.parameters(), fm.parameters()):
                q.copy_(src)
        trees.append(t)
    w = [float(x) for x in np.random.default_rng(16).dirichlet(np.ones(16))]

    def e2e():
        fa.FedAvg.aggregate(trees, w)
        torch.cuda.synchronize()

    row = {"peers": 16, "params": p, "dtype": "bf16", "modules": len(list(trees[0].modules())),
           "tensors": len(list(trees[0].parameters())), "end_to_end_ms": _median_ms(e2e, reps),
           "layout_walk_ms": _median_ms(lambda: fa._device_layout(trees), reps)}
    got, want = fa.FedAvg.aggregate(trees, w), fa.FedAvg.aggregate(flat, w)
    torch.cuda.synchronize()
    row["parity_ok"] = all(torch.equal(a.detach().view(torch.int16), b.detach().view(torch.int16))
                           for a, b in zip(got.parameters(), want.parameters()))
    row["parity"] = "every parameter of the tree round's result == the ParameterList round's, bit for bit"
    del flat, trees, got, want
    torch.cuda.empty_cache()
    return row


def cpu_layout_configs(budget_s=2.0):
    """The reference op sequence (oracle port of fedavg.py:13-26, torch-CPU, T tensors per
    model) on the pageable modules of host_inclusive_configs."""
    sys.path.insert(0, ROOT)
    from oracle.fedavg_oracle import fedavg_modules_torch  # timed CPU baseline (kind "port")

    torch.set_num_threads(cpu_threads()[0])
    res = {}
    for name, (lay, n, dts) in HOST_CONFIGS.items():
        dt = torch.float32 if dts == "f32" else torch.bfloat16
        models, p = _layout_models(lay, n, dt, False)
        w = [float(1.0 / n)] * n
        ts = []
        start = time.perf_counter()
        while (time.perf_counter() - start < budget_s and len(ts) < 20) or len(ts) < 1:
            t0 = time.perf_counter()
            fedavg_modules_torch(models, w)
            ts.append(time.perf_counter() - t0)
        res[name] = {"cpu_port_ms": round(statistics.median(ts) * 1e3, 2), "reps": len(ts)}
        del models
    return res


def host_inclusive_small(reps=50):
    """The reference's most frequent call: FedAvg.aggregate on small CPU models (GNLeNet,
    configs[1]; GL merges N=2 every round, DFL N=8), end to end (per-call overhead, not
    bandwidth, decides here; the torch-CPU op sequence on the same modules is timed in the
    cpu_baseline leg)."""
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg

    out = {}
    for layers in (False, True):
        for n in (2, 8):
            models = _gnlenet_models(n, layers)
            w = [float(1.0 / n)] * n
            out["gnlenet%s_n%d" % ("_layers" if layers else "", n)] = {
                "ours_ms": _median_ms(lambda: FedAvg.aggregate(models, w), reps)}
    return out


def wire_ingress(p, device, reps=5):
    """§8 f1: one peer's serialize_model bytes (25 M fp32) -> HBM PeerSlab row, against the
    reference's decode (pickle.loads, which also runs a torch.load per storage)."""
    import pickle

    from torch import nn

    from accdfl_amd.core import wire
    from accdfl_amd.core.peer_slab import PeerSlab

    m = nn.Module()
    m.w = nn.Parameter(torch.randn(p, generator=torch.Generator().manual_seed(7)) * 0.05)
    data = wire.serialize_model(m)
    slab = PeerSlab([(p,)], torch.float32, capacity=1, device=device)

    def ours():
        slab.reset()
        slab.stage(wire.parameter_tensors(wire.loads_state_dict(data, copy=False), m))
        slab.copy_stream.synchronize()

    def ref_decode():
        pickle.loads(data)  # bytes this process made: the reference's unserialize step

    out = {}
    for name, fn in (("ours_decode_and_stage_ms", ours), ("reference_pickle_loads_ms", ref_decode)):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        out[name] = round(statistics.median(ts) * 1e3, 2)
    out["payload_MB"] = round(len(data) / 1e6, 1)
    out["ours_GBps"] = round(len(data) / (out["ours_decode_and_stage_ms"] / 1e3) / 1e9, 1)
    return out


EVA_BLOCK = 60_000  # accdfl/core/session_settings.py:76 (eva block_size)


def dfl_messages(n, p, seed=300):
    """n DFL 'trained_model' messages of a p-parameter fp32 model as EVA delivers them: the
    blocks of serialize_model bytes + the pickled population view (accdfl/dfl/community.py:
    478-509 builds them), with each message's model_data_len."""
    import pickle

    from torch import nn

    from accdfl_amd.core import wire

    msgs = []
    for k in range(n):
        m = nn.Module()
        m.w = nn.Parameter(torch.randn(p, generator=torch.Generator().manual_seed(seed + k)) * 0.05)
        mb = wire.serialize_model(m)
        view = pickle.dumps({"peer%d" % j: j for j in range(16)})
        msgs.append((wire.payload_blocks(mb + view, EVA_BLOCK), len(mb)))
    return msgs


def dfl_round(msgs, p, device, reps=3):
    """§8 f1-f3 at north-star scale: one DFL aggregator round (accdfl/dfl/community.py:576-673)
    end to end — every message's EVA blocks split at model_data_len and decoded into page-locked
    ingress buffers -> HBM PeerSlab tiles (no b''.join, no slice copy, no create_model /
    load_state_dict), the uniform average (:673), and its serialize_model bytes (:556-567).
    ``phases`` splits the ingress (sums over the round's peers, medians over the reps): the wire
    split, decode + gather into the page-locked buffers (of which the native gather), the stage
    calls, the copy stream's own time for the peers' H2D (HIP events, ``copy_busy_ms``) and its idle
    time between them, and ``wait_ms``: the copy stream draining after the loop (ingress_complete_ms =
    ingress_ms + wait_ms: when the last peer is in HBM)."""
    from torch import nn

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager
    from types import SimpleNamespace

    n = len(msgs)
    template = nn.Module()
    template.w = nn.Parameter(torch.zeros(p))
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0,
                            capacity=n, template=template, device=device)

    def one():
        mm.reset_incoming_trained_models()
        ph = mm.start_phases()
        wire.GATHER_MS = []
        t_split = 0.0
        t0 = time.perf_counter()
        for k, (blocks, ml) in enumerate(msgs):
            ts = time.perf_counter()
            head, _ = wire.split_blocks(blocks, ml)
            t_split += time.perf_counter() - ts
            mm.process_incoming_serialized(b"peer%d" % k, head)
        t1 = time.perf_counter()
        mm.slab.copy_stream.synchronize()
        tw = time.perf_counter()
        gathers, wire.GATHER_MS = wire.GATHER_MS, None
        mm.phases = None
        ev = ph["copy_events"]
        busy = sum(a.elapsed_time(b) for a, b in ev)
        idle = sum(ev[i - 1][1].elapsed_time(ev[i][0]) for i in range(1, len(ev)))
        phases = {"split_ms": t_split * 1e3, "decode_gather_ms": sum(ph["decode_gather_ms"]),
                  "native_gather_ms": sum(gathers), "stage_issue_ms": sum(ph["stage_issue_ms"]),
                  "copy_busy_ms": busy, "copy_idle_between_peers_ms": idle, "wait_ms": (tw - t1) * 1e3}
        out = mm.aggregate_trained_models()
        t2 = time.perf_counter()
        data = wire.serialize_model(out)
        t3 = time.perf_counter()
        assert len(data) > p * 4
        # the same average as bytes straight from HBM (aggregate_serialized: no result module)
        t4 = time.perf_counter()
        direct = mm.aggregate_serialized()
        t5 = time.perf_counter()
        assert len(direct) == len(data)
        return (t1 - t0, t2 - tw, t3 - t2, t3 - t0, t5 - t4, tw - t0), phases

    one()
    runs = [one() for _ in range(reps)]
    med = [statistics.median(r[0][i] for r in runs) for i in range(6)]
    phases = {k: round(statistics.median(r[1][k] for r in runs), 2) for k in runs[0][1]}
    h2d_bytes = n * p * 4
    phases["copy_GBps"] = round(h2d_bytes / (phases["copy_busy_ms"] / 1e3) / 1e9, 2) if phases["copy_busy_ms"] else None
    phases["gather_GBps"] = (round(h2d_bytes / (phases["native_gather_ms"] / 1e3) / 1e9, 2)
                             if phases["native_gather_ms"] else None)
    return {"peers": n, "params": p, "eva_block_bytes": EVA_BLOCK,
            "ingress_ms": round(med[0] * 1e3, 2), "ingress_complete_ms": round(med[5] * 1e3, 2),
            "aggregate_ms": round(med[1] * 1e3, 2),
            "egress_serialize_ms": round(med[2] * 1e3, 2), "round_ms": round(med[3] * 1e3, 2),
            "round_GBps": round((n + 1) * p * 4 / med[3] / 1e9, 2),
            "aggregate_serialized_ms": round(med[4] * 1e3, 2),
            "phases": phases,
            "aggregate_serialized_path": "DeviceModelManager.aggregate_serialized: the reduce, then the averaged row "
                                         "D2H in 32 MiB chunks through page-locked bounce buffers straight into "
                                         "the payload bytes (no result module; replaces aggregate + serialize)",
            "path": "EVA blocks -> split at model_data_len -> restricted decode, gather into page-locked ingress "
                    "buffers -> one 2D H2D per peer straight into the tile-interleaved PeerSlab (dla_slab_stage) "
                    "-> reduce -> D2H into the pooled result -> serialize_model bytes"}


def dfl_round_layout(name, n, dt, device, reps=3):
    """§8 f1-f3 on a real many-tensor layout: the DFL aggregator round of ``n`` models of ``name``
    (e.g. configs[4]'s google_speech ResNet-34, 110 parameter tensors and 108 BN buffers in bf16)
    arriving as EVA blocks of their serialize_model bytes — most tensors cross the 60 000-byte blocks,
    so each is gathered into the peer's page-locked ingress buffer at its own offset and sent to its
    PeerSlab tiles — then the average as serialize_model bytes straight from HBM
    (aggregate_serialized).  ``parity_ok``: every parameter of the decoded payload equals
    FedAvg.aggregate on the same modules (the device path, no wire), bit for bit."""
    import pickle
    from types import SimpleNamespace

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.gradient_aggregation.fedavg import FedAvg
    from accdfl_amd.core.model_manager import DeviceModelManager

    models, p = _layout_models(name, n, dt, pinned=False, seed=4200)
    view = pickle.dumps({"peer%d" % j: j for j in range(16)})
    msgs = []
    for m in models:
        mb = wire.serialize_model(m)
        msgs.append((wire.payload_blocks(mb + view, EVA_BLOCK), len(mb)))
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0,
                            capacity=n, template=models[0], device=device)
    w = [float(x) for x in np.random.default_rng(n).dirichlet(np.ones(n))]

    def one():
        mm.reset_incoming_trained_models()
        t0 = time.perf_counter()
        for k, (blocks, ml) in enumerate(msgs):
            head, _ = wire.split_blocks(blocks, ml)
            mm.process_incoming_serialized(b"peer%d" % k, head)
        t1 = time.perf_counter()
        mm.slab.copy_stream.synchronize()
        t2 = time.perf_counter()
        data = mm.aggregate_serialized(w)
        t3 = time.perf_counter()
        return (t1 - t0, t2 - t0, t3 - t2, t3 - t0), data

    one()
    runs = [one() for _ in range(reps)]
    med = [statistics.median(r[0][i] for r in runs) for i in range(4)]
    got = wire.loads_state_dict(runs[-1][1])
    dev_models = [m.to(device) for m in models]
    want = FedAvg.aggregate(dev_models, w)
    torch.cuda.synchronize()
    names = [k for k, _ in want.named_parameters()]
    ok = all(torch.equal(got[k].view(torch.int16 if dt != torch.float32 else torch.int32),
                         v.detach().cpu().view(torch.int16 if dt != torch.float32 else torch.int32))
             for k, v in zip(names, want.parameters()))
    in_bytes = n * p * torch.empty((), dtype=dt).element_size()
    n_cross = sum(1 for s in _layout(name)[0] if int(np.prod(s) if s else 1) * torch.empty((), dtype=dt).element_size()
                  >= EVA_BLOCK)
    native = all(getattr(v, "_sd", 0) is None for v in list(mm.incoming_trained_models.values())[1:])
    # the per-peer phase split of one more round (decode = native scan + batched gather, stage = the call
    # that enqueues the peer's copy; copy_busy: the copy stream's own time for the peers' H2D)
    mm.reset_incoming_trained_models()
    ph = mm.start_phases()
    for k, (blocks, ml) in enumerate(msgs):
        head, _ = wire.split_blocks(blocks, ml)
        mm.process_incoming_serialized(b"peer%d" % k, head)
    mm.slab.copy_stream.synchronize()
    mm.phases = None
    busy = sum(a.elapsed_time(b) for a, b in ph["copy_events"])
    phases = {"decode_gather_ms": round(sum(ph["decode_gather_ms"]), 2),
              "stage_issue_ms": round(sum(ph["stage_issue_ms"]), 2), "copy_busy_ms": round(busy, 2),
              "copy_GBps": round(in_bytes / (busy / 1e3) / 1e9, 2) if busy else None}
    ref = dfl_round_layout_reference_style(msgs, _layout_models(name, 1, dt, pinned=False, seed=4200)[0][0])
    return {"layout": name, "peers": n, "params": p, "parameter_tensors": len(names), "dtype": str(dt),
            "eva_block_bytes": EVA_BLOCK, "tensors_of_at_least_one_block": n_cross,
            "ingress_ms": round(med[0] * 1e3, 2), "ingress_complete_ms": round(med[1] * 1e3, 2),
            "ingress_GBps": round(in_bytes / med[1] / 1e9, 2),
            "aggregate_serialized_ms": round(med[2] * 1e3, 2), "round_ms": round(med[3] * 1e3, 2),
            "native_ingress": native, "phases": phases,
            "reference_style_ingress_ms": ref,
            "ingress_speedup_vs_reference_style": round(ref / (med[1] * 1e3), 1) if ref else None,
            "parity_ok": bool(ok),
            "parity": "every parameter of the decoded aggregate_serialized payload == FedAvg.aggregate on the same "
                      "modules on the device (no wire), bit for bit",
            "path": "EVA blocks -> split at model_data_len -> native scan of the state-dict pickle (csrc/walk.cpp) -> "
                    "ONE batched gather of every storage into the page-locked ingress buffer, parameters back to "
                    "back -> ONE 2D H2D per peer into the tile-interleaved PeerSlab -> reduce -> payload bytes "
                    "from HBM (aggregate_serialized)"}


def dfl_round_layout_reference_style(msgs, template, reps=2):
    """The same many-tensor ingress the reference's way, on this host's CPU, for the same payloads:
    b''.join of the EVA blocks (accdfl/util/eva/transfer/incoming.py:35), the model_data_len slice
    (accdfl/dfl/community.py:587), pickle.loads + load_state_dict into a fresh model
    (accdfl/core/models/__init__.py:13-16; create_model's allocation stood for by a deepcopy of the
    template).  Median ms for all peers (bytes this process made: pickle.loads is the reference's)."""
    import copy
    import pickle

    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for blocks, ml in msgs:
            data = b"".join(blocks)
            m = copy.deepcopy(template)
            m.load_state_dict(pickle.loads(data[:ml]))
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e3, 1)


def dfl_round_reference_style(msgs, p, reps=2):
    """The same round the way the reference runs it, on this host's CPU: b''.join of the EVA
    blocks (accdfl/util/eva/transfer/incoming.py:35), the model_data_len slice
    (accdfl/dfl/community.py:587), pickle.loads + load_state_dict into a fresh model
    (accdfl/core/models/__init__.py:13-16), the FedAvg op sequence (oracle port of fedavg.py:
    13-26), serialize_model.  Timed CPU comparison only."""
    import copy
    import pickle

    from torch import nn

    sys.path.insert(0, ROOT)
    from oracle.fedavg_oracle import fedavg_modules_torch  # timed CPU comparison (kind "port")
    from accdfl_amd.core import wire

    template = nn.Module()
    template.w = nn.Parameter(torch.zeros(p))

    def one():
        t0 = time.perf_counter()
        models = []
        for blocks, ml in msgs:
            data = b"".join(blocks)
            model_bytes = data[:ml]
            m = copy.deepcopy(template)
            m.load_state_dict(pickle.loads(model_bytes))  # bytes this process made
            models.append(m)
        t1 = time.perf_counter()
        out = fedavg_modules_torch(models, None)
        t2 = time.perf_counter()
        wire.serialize_model(out)
        t3 = time.perf_counter()
        return t1 - t0, t2 - t1, t3 - t2, t3 - t0

    runs = [one() for _ in range(reps)]
    med = [statistics.median(r[i] for r in runs) for i in range(4)]
    return {"ingress_ms": round(med[0] * 1e3, 1), "aggregate_ms": round(med[1] * 1e3, 1),
            "egress_serialize_ms": round(med[2] * 1e3, 1), "round_ms": round(med[3] * 1e3, 1),
            "threads": torch.get_num_threads()}


def _cpu_port_ms(n, share, dt, budget_s=1.5, max_elems=500_000_000):
    """The reference op sequence (oracle/fedavg_oracle.py, torch-CPU, product temporary held) on the same share,
    on this host's cores: median ms of a bounded sample, or None above max_elems."""
    if n * share > max_elems:
        return None, 0
    sys.path.insert(0, ROOT)
    from oracle.fedavg_oracle import fedavg_flat_torch_warm  # timed CPU baseline (kind "port")

    threads = cpu_threads()[0]
    torch.set_num_threads(threads)
    base = torch.randn(share, generator=torch.Generator().manual_seed(1000)) * 0.05
    peers = [(base * (1.0 + 0.01 * k)).to(dt) for k in range(n)]  # values do not change CPU time
    w = [float(1.0 / n)] * n
    out = torch.empty(share, dtype=dt)
    tmp = torch.empty(share, dtype=dt)
    fedavg_flat_torch_warm(peers, w, out, tmp)
    ts = []
    start = time.perf_counter()
    while (time.perf_counter() - start < budget_s and len(ts) < 50) or len(ts) < 3:
        t0 = time.perf_counter()
        fedavg_flat_torch_warm(peers, w, out, tmp)
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3, threads


def time_graph(launch, per_graph=20, reps=10):
    """Seconds per launch with `per_graph` launches captured in one HIP graph and replayed
    `reps` times: the device-side cost of a reduce without the host's per-launch overhead
    (which bounds back-to-back eager launches of a few-microsecond kernel)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        launch(s.cuda_stream)  # warm
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        sp = torch.cuda.current_stream().cuda_stream
        for _ in range(per_graph):
            launch(sp)
    g.replay()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        g.replay()
    ev1.record()
    torch.cuda.synchronize()
    del g
    return ev0.elapsed_time(ev1) / 1e3 / (reps * per_graph)


def baseline_configs(device, steps=40):
    """Device-resident reduce rate of each BASELINE config's per-GPU share staged as PeerSlab
    holds it (SlabInput, a prepared launch; bytes = (N + 1) * share * sizeof).  The reference
    op sequence on the same shares is timed in the cpu_baseline leg (cpu_per_config) and the
    ratio filled in as gpu_over_cpu."""
    from accdfl_amd import _lib

    res = {}
    for name, (n, params, dts, gpus) in CONFIGS.items():
        dt = torch.float32 if dts == "f32" else torch.bfloat16
        es = 4 if dts == "f32" else 2
        share = -(-params // gpus)
        inp = SlabInput(n, share, dt, device, 1000, [float(1.0 / n)] * n)
        sp = torch.cuda.current_stream().cuda_stream
        # median of 5 timed runs of `steps` launches, the first after the settle phase
        ev = statistics.median(time_kernel(lambda: inp.launch(sp), steps, 10, 1, settle_s=None if i == 0 else 0)[1]
                               for i in range(5))
        tg = time_graph(inp.launch)
        byts = (n + 1) * share * es
        res[name] = {"peers": n, "params_per_gpu": share, "dtype": dts, "us_per_reduce": round(ev / steps * 1e6, 2),
                     "GB/s": round(byts / (ev / steps) / 1e9, 1), "bytes": byts,
                     "us_per_reduce_graph": round(tg * 1e6, 2), "GB/s_graph": round(byts / tg / 1e9, 1),
                     "regime": "HBM" if byts > 256 << 20 else "Infinity-Cache / launch-latency",
                     "kernel": inp.kernel}
        del inp
        torch.cuda.empty_cache()
    return res


def cpu_per_config():
    """The reference op sequence (oracle port, torch-CPU) on every BASELINE config's per-GPU
    share, on this host's CPU share (flat, one tensor per peer: a lower bound on the
    reference's per-tensor loop, which pays T dispatches per peer)."""
    res = {}
    for name, (n, params, dts, gpus) in CONFIGS.items():
        dt = torch.float32 if dts == "f32" else torch.bfloat16
        es = 4 if dts == "f32" else 2
        share = -(-params // gpus)
        ms, threads = _cpu_port_ms(n, share, dt)
        if ms is not None:
            res[name] = {"cpu_port_ms": round(ms, 3), "cpu_port_GB/s": round((n + 1) * share * es / (ms / 1e3) / 1e9, 2),
                         "cpu_threads": threads}
    return res


def cpu_baseline_all(args, result, n, p, headline=None):
    """The cpu_baseline object: the reference op sequence on the host cores (the only leg that runs
    the oracle port), plus every other CPU comparison, each ratio filled into the GPU row it
    belongs to.  ``headline``: see cpu_baseline."""
    cb = cpu_baseline(n, p, args.cpu_seconds, headline)
    if not args.no_small:
        cb["per_config"] = cpu_per_config()
        for name, row in cb["per_config"].items():
            g = result.get("baseline_configs", {}).get(name)
            if g:
                g["gpu_over_cpu"] = round(row["cpu_port_ms"] * 1e3 / g["us_per_reduce"], 1)
    if not args.no_host_inclusive:
        cb["gnlenet_small"] = cpu_gnlenet_small()
        for key, row in cb["gnlenet_small"].items():
            result.get("host_inclusive_small", {}).get(key, {})["cpu_port_ms"] = row["cpu_port_ms"]
        msgs = dfl_messages(n, p)
        cb["dfl_round_reference_style"] = dfl_round_reference_style(msgs, p)
        del msgs
        log("cpu baseline: reference op sequence on the config layouts")
        cb["layout_configs"] = cpu_layout_configs()
        for name, row in cb["layout_configs"].items():
            g = result.get("host_inclusive_configs", {}).get(name)
            if g and "pageable_ms" in g:
                g["cpu_port_ms"] = row["cpu_port_ms"]
                g["pageable_over_cpu"] = round(row["cpu_port_ms"] / g["pageable_ms"], 1)
                if g.get("staged_on_arrival_ms"):
                    g["staged_over_cpu"] = round(row["cpu_port_ms"] / g["staged_on_arrival_ms"], 1)
    return cb


def cpu_gnlenet_small(reps=50):
    """The torch-CPU op sequence (oracle port of fedavg.py:13-26) on the GNLeNet rounds of
    host_inclusive_small."""
    sys.path.insert(0, ROOT)
    from oracle.fedavg_oracle import fedavg_modules_torch  # timed CPU baseline (kind "port")

    out = {}
    for layers in (False, True):
        for n in (2, 8):
            models = _gnlenet_models(n, layers)
            w = [float(1.0 / n)] * n
            out["gnlenet%s_n%d" % ("_layers" if layers else "", n)] = {
                "cpu_port_ms": _median_ms(lambda: fedavg_modules_torch(models, w), reps)}
    return out


# Fixed models for the strong-scaling lines: (peers, params of the whole model, dtype).
STRONG = {
    "north star, 8 peers x 25 M f32": (8, NS_PARAMS, "f32"),
    "configs[3] CIFAR-10 GNLeNet, 64 peers": (64, 85_354, "f32"),
    "configs[3'] CIFAR-10 ResNet-8, 64 peers": (64, 4_932_344, "f32"),
    "configs[4] google_speech ResNet-34, 128 peers, bf16": (128, 21_296_355, "bf16"),
}
_MALL_BYTES = 256 << 20
_ROTATE_BYTES = 1 << 30


def strong_line(legs, name, rank, world, device, steps, warmup):
    """STRONG model `name` split into ``world`` contiguous 256-B-aligned parameter buckets
    (core/sharding.bucket_bounds, the bucket-sharded layout of SURVEY.md §8e); rank r reduces
    bucket r of every peer.  Whole-model algorithmic bytes / max-over-ranks step time.  Each
    rank cycles through enough copies of its bucket that the working set is >= 1 GiB, so a
    small bucket cannot be served from the 256 MiB Infinity Cache step after step
    ("cache_warm" repeats one copy, for comparison).  At N > 1 the all-gather that reassembles
    the whole averaged model on every rank (RCCL) is timed separately (never inside the line),
    on the ranks' real averaged buckets, and the reassembled model is checked bit for bit on rank 0
    against ONE reduce of the whole model rebuilt from the same seeds (copy 0 of rank r's bucket:
    seed 1000 + 7 r + k)."""
    from accdfl_amd.core import wsum
    from accdfl_amd.core.sharding import BucketShardedFedAvg, bucket_bounds

    n, params, dts = STRONG[name]
    dt = torch.float32 if dts == "f32" else torch.bfloat16
    es = 4 if dts == "f32" else 2
    bounds = bucket_bounds(params, world, 256 // es)
    s0, e0 = bounds[rank]
    m = max(e0 - s0, 0)
    pitch = max(128, (m + 127) // 128 * 128)
    set_bytes = (n + 1) * pitch * es
    copies = 1 if set_bytes >= _ROTATE_BYTES else min(64, -(-_ROTATE_BYTES // set_bytes))
    w = [float(x) for x in np.random.default_rng(0).dirichlet(np.ones(n))]
    ref = None
    if world > 1 and rank == 0:  # the single-GPU reference of the whole model (built before the timing)
        full = torch.empty((n, params), dtype=dt, device=device)
        for r, (s, e) in enumerate(bounds):
            if e > s:
                pr = max(128, (e - s + 127) // 128 * 128)
                full[:, s:e].copy_(make_slab(n, pr, dt, device, 1000 + 7 * r)[:, : e - s])
        ref = wsum.wsum(list(full), w)
        del full
        torch.cuda.empty_cache()
    one_gpu_s = None
    if world > 1 and rank == 0:
        # the same whole model reduced on ONE GPU in the same run (rank 0's, the other GPUs idle), laid
        # out and rotated as the N = 1 line does it: the in-run reference of the strong speedup
        pw = max(128, (params + 127) // 128 * 128)
        wcopies = 1 if (n + 1) * pw * es >= _ROTATE_BYTES else min(64, -(-_ROTATE_BYTES // ((n + 1) * pw * es)))
        whole = [SlabInput(n, params, dt, device, 1000 + 131 * c, w) for c in range(wcopies)]
        wctr = [0]

        def step_whole():
            whole[wctr[0] % len(whole)].launch(torch.cuda.current_stream().cuda_stream)
            wctr[0] += 1
        wall1, _ = time_kernel(step_whole, steps, warmup, 1)
        one_gpu_s = wall1 / steps
        del whole
        torch.cuda.empty_cache()
    inputs = [SlabInput(n, m, dt, device, 1000 + 131 * c + 7 * rank, w) for c in range(copies)] if m else []
    sp = torch.cuda.current_stream().cuda_stream
    ctr = [0]

    def step_rot():
        if inputs:
            inputs[ctr[0] % len(inputs)].launch(sp)
        ctr[0] += 1

    def step_warm():  # last: leaves copy 0's average in inputs[0].out
        if inputs:
            inputs[0].launch(sp)

    legs.go()
    wall, ev = time_kernel(step_rot, steps, warmup, world)
    wall_w, _ = time_kernel(step_warm, steps, warmup, world)
    total = (n + 1) * params * es
    row = {"peers": n, "params": params, "dtype": dts, "buckets": world,
           "bucket_params_max": max(e - s for s, e in bounds),
           "ms_per_step": round(wall / steps * 1e3, 5),
           "value": round(total / (wall / steps) / 1e9, 2), "unit": "GB/s",
           "kernel_us_max_rank": round(ev / steps * 1e6, 2),
           "input_copies_rotated": copies,
           "cache_warm_value": round(total / (wall_w / steps) / 1e9, 2),
           "regime": "HBM" if (n + 1) * (bounds[0][1] - bounds[0][0]) * es > _MALL_BYTES
           else "bucket fits the Infinity Cache; rotated copies keep it HBM-resident",
           "kernel": inputs[0].kernel if inputs else None}
    if world > 1:
        cdev = _comm_device(device)
        sh = BucketShardedFedAvg(params, dt, device=cdev)
        bucket = torch.zeros(sh.bucket_len, dtype=dt, device=cdev)
        if m:
            bucket[:m].copy_(inputs[0].out[:m])
        full = torch.empty(params, dtype=dt, device=cdev)
        wall_g, _ = time_kernel(lambda: sh.all_gather(bucket, full), 10, 2, world, settle_s=0)
        legs.settled()
        row["allgather_ms"] = round(wall_g / 10 * 1e3, 4)
        row["with_allgather_value"] = round(total / (wall / steps + wall_g / 10) / 1e9, 2)
        if rank == 0:
            row["parity_ok"] = same_bits(full.to(device), ref)
            row["one_gpu_ms_per_step"] = round(one_gpu_s * 1e3, 5)
            row["one_gpu_value"] = round(total / one_gpu_s / 1e9, 2)
            row["speedup_vs_one_gpu"] = round(one_gpu_s / (wall / steps), 3)
            row["efficiency"] = round(one_gpu_s / (wall / steps) / world, 3)
            row["speedup_with_allgather"] = round(one_gpu_s / (wall / steps + wall_g / 10), 3)
    del inputs
    torch.cuda.empty_cache()
    return row


def dry_run(args, rank, world, cpu_group):
    """No GPU: the launch, the rendezvous, the rank-count check, the bucket split the
    strong-scaling lines use and a gloo all-gather leg with its parity check, all through the
    Legs runner (agreed skips, fatal exits, the watchdog); rank 0 prints one JSON line (checked by
    the CPU tests, which also inject failures with BENCH_INJECT_FAIL)."""
    from accdfl_amd.core.sharding import bucket_bounds

    result = {"dry_run": True, "n_gpus": world, "launch": launch_info(world)}
    legs = Legs(rank, world, cpu_group, args.leg_timeout, result)

    def rendezvous(L):
        mine = {name: list(bucket_bounds(params, world, 256 // (4 if dts == "f32" else 2))[rank])
                for name, (_, params, dts) in STRONG.items()}
        got = [mine]
        L.go()
        if world > 1:
            got = [None] * world
            dist.all_gather_object(got, mine)
        L.settled()
        buckets = {name: [g[name] for g in got] for name in STRONG}
        cover = all(b[0][0] == 0 and b[-1][1] == STRONG[name][1] and all(x[1] == y[0] for x, y in zip(b, b[1:]))
                    for name, b in buckets.items())
        return {"buckets": buckets, "parity_ok": cover}

    def gloo_allgather(L, length=100_003):
        mine = _rank_content(rank, length, torch.float32, torch.device("cpu"))
        L.go()
        got = gather_all(mine, length, torch.device("cpu")) if world > 1 else [mine]
        L.settled()
        want = [_rank_content(r, length, torch.float32, torch.device("cpu")) for r in range(world)]
        return {"elems_per_rank": length, "parity_ok": all(same_bits(a, b) for a, b in zip(got, want))}

    def strong_gather(L, name, scale=64):
        # the strong line's exchange without a GPU: every rank's bucket of the fixed model (1/scale of
        # its parameters, same split rule), filled with rank-seeded content, all-gathered over gloo and
        # checked element for element against the whole model rebuilt from the seeds
        n_, params, dts = STRONG[name]
        small = max(1, params // scale)
        bounds = bucket_bounds(small, world, 256 // (4 if dts == "f32" else 2))
        s_, e_ = bounds[rank]
        mine = _rank_content(rank, max(e_ - s_, 0), torch.float32, torch.device("cpu"))
        L.go()
        t0 = time.perf_counter()
        got = gather_all(mine, max(e - s for s, e in bounds), torch.device("cpu")) if world > 1 else [mine]
        ms = (time.perf_counter() - t0) * 1e3
        L.settled()
        ok = all(same_bits(g[: e - s], _rank_content(r, e - s, torch.float32, torch.device("cpu")))
                 for r, (g, (s, e)) in enumerate(zip(got, bounds)))
        return {"buckets": world, "params_scaled": small, "allgather_ms_gloo": round(ms, 3), "parity_ok": ok,
                "value": None, "speedup_vs_one_gpu": None, "efficiency": None}

    rows = {"rendezvous": legs.run("rendezvous", rendezvous), "gloo_allgather": legs.run("gloo_allgather",
                                                                                          gloo_allgather)}
    strong = {"scaling": "strong", "n_gpus": world, "dry_run": "bucket split + gloo all-gather of scaled models; "
                                                               "no GPU, so no rates"}
    for key, name in (("north_star", "north star, 8 peers x 25 M f32"),
                      ("configs3_resnet8", "configs[3'] CIFAR-10 ResNet-8, 64 peers"),
                      ("configs4_resnet34_bf16", "configs[4] google_speech ResNet-34, 128 peers, bf16")):
        strong[key] = legs.run("strong: " + name, strong_gather, name)
    result["strong_headline"] = strong
    result["buckets"] = rows["rendezvous"].pop("buckets", None)
    result["legs"] = rows
    result["legs_failed"] = legs.failed
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def sweep(args, device):
    from accdfl_amd import _lib
    from accdfl_amd.core import wsum

    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}[args.dtype]
    es = {"f32": 4, "f64": 8}.get(args.dtype, 2)
    slab = make_slab(args.peers, (args.params + 127) // 128 * 128, dt, device, 1000)  # 16-B aligned rows
    out = torch.empty(args.params, dtype=dt, device=device)
    w = [float(1.0 / args.peers)] * args.peers
    ptrs = [slab[k].data_ptr() for k in range(args.peers)]
    code = wsum.dtype_code(dt)
    sp = torch.cuda.current_stream().cuda_stream
    if args.sweep_cfgs:
        cfgs = [tuple(int(x) for x in item.split(",")) for item in args.sweep_cfgs.split(";") if item]
    else:
        cfgs = [(v, c, 0, b) for v in (1, 2, 4) for c in (1, 2, 4) for b in (64, 256)]
    if args.pads:
        byts = (args.peers + 1) * args.params * es
        pads = [int(x) for x in args.pads.split(",")]
        del slab
        res = {}
        for rnd in range(5):
            for pad in pads:
                pitch = (args.params * es + pad + 15) // 16 * 16 // es
                sl = make_slab(args.peers, pitch, dt, device, 1000)
                pp = [sl[k].data_ptr() for k in range(args.peers)]
                fn = lambda: _lib.wsum_ptrs(code, pp, w, args.params, out.data_ptr(), sp)  # noqa: E731
                _, ev = time_kernel(fn, 50, 5, 1, settle_s=0.02)
                res.setdefault(pad, []).append(ev / 50)
                del sl
                torch.cuda.empty_cache()  # fresh physical pages for the next allocation
        for t, pad in sorted((statistics.median(v), k) for k, v in res.items()):
            print(json.dumps({"pad_bytes": pad, "us": round(t * 1e6, 2), "GB/s": round(byts / t / 1e9, 1)}))
        return
    if args.tile_bytes:
        byts = (args.peers + 1) * args.params * es
        tiles = [int(x) for x in args.tile_bytes.split(",")]
        slabs = {}
        for tb in tiles:
            te = tb // es
            n_t = -(-args.params // te)
            slabs[tb] = make_slab(n_t * args.peers, te, dt, device, 2000)  # [n_tiles * N, T] = [n_tiles][N][T]
        res = {}
        variants = [int(x) for x in (args.sweep_cfgs.split(",") if args.sweep_cfgs else ["9", "12", "21"])]
        for rnd in range(5):
            fn = lambda: _lib.wsum_ptrs(code, ptrs, w, args.params, out.data_ptr(), sp)  # noqa: E731
            _, ev = time_kernel(fn, 50, 5, 1, settle_s=0.02)
            res.setdefault(("row-major default", 0), []).append(ev / 50)
            for tb in tiles:
                for v in variants:
                    cfg = _lib.LaunchCfg(v, 0, 0, 0)
                    fn = lambda: _lib.wsum_slab_tiled_ptr(code, slabs[tb].data_ptr(), tb // es, args.peers, w,  # noqa
                                                          args.params, out.data_ptr(), sp, cfg)
                    _, ev = time_kernel(fn, 50, 5, 1, settle_s=0.02)
                    res.setdefault(("tiled %d B" % tb, v), []).append(ev / 50)
        for t, k in sorted((statistics.median(v), k) for k, v in res.items()):
            print(json.dumps({"layout": k[0], "variant": k[1], "us": round(t * 1e6, 2),
                              "GB/s": round(byts / t / 1e9, 1), "min_us": round(min(res[k]) * 1e6, 2)}))
        return
    if args.libs:
        import ctypes

        libs = []
        for path in args.libs.split(","):
            so = ctypes.CDLL(os.path.abspath(path))
            so.dla_wsum_ex.argtypes = _lib.lib().so.dla_wsum_ex.argtypes
            libs.append((os.path.basename(path), so))
        pa = _lib._ptr_array(ptrs)
        wa = _lib._dbl_array(w)
        res = {(name,) + c: [] for name, _ in libs for c in cfgs}
        for rnd in range(7):
            for name, so in libs:
                for c in cfgs:
                    cfg = _lib.LaunchCfg(*c)
                    fn = lambda: so.dla_wsum_ex(code, pa, wa, len(ptrs), args.params, out.data_ptr(), sp,  # noqa
                                                ctypes.byref(cfg))
                    _, ev = time_kernel(fn, 50, 5, 1, settle_s=0.02)
                    res[(name,) + c].append(ev / 50)
        byts = (args.peers + 1) * args.params * es
        for t, k in sorted((statistics.median(v), k) for k, v in res.items()):
            print(json.dumps({"lib": k[0], "cfg": k[1:], "us": round(t * 1e6, 2),
                              "GB/s": round(byts / t / 1e9, 1), "min_us": round(min(res[k]) * 1e6, 2)}))
        return
    res = {c: [] for c in cfgs}
    for rnd in range(5):
        for c in cfgs:
            cfg = _lib.LaunchCfg(*c)
            fn = lambda: _lib.wsum_ptrs(code, ptrs, w, args.params, out.data_ptr(), sp, cfg)  # noqa: E731
            _, ev = time_kernel(fn, 50, 5, 1, settle_s=0.02)
            res[c].append(ev / 50)
    byts = (args.peers + 1) * args.params * es
    # in place: the average overwrites peer 0's row (allowed by the ABI: out may alias peers[0])
    for c in ([] if args.sweep_cfgs else [(4, 1, 0, 64)]):
        cfg = _lib.LaunchCfg(*c)
        key = (c[0], c[1], -1, c[3])
        res[key] = []
        for rnd in range(5):
            fn = lambda: _lib.wsum_ptrs(code, ptrs, w, args.params, ptrs[0], sp, cfg)  # noqa: E731
            _, ev = time_kernel(fn, 50, 5, 1, settle_s=0.02)
            res[key].append(ev / 50)
    rows = sorted(((statistics.median(v), c) for c, v in res.items()))
    for t, c in rows:
        print(json.dumps({"variant": c[0], "chunks": c[1], "grid": c[2], "block": c[3] if len(c) > 3 else 0,
                          "us": round(t * 1e6, 2),
                          "GB/s": round(byts / t / 1e9, 1), "min_us": round(min(res[c]) * 1e6, 2)}))
    del slab
    if not args.no_ceilings:
        for k, v in measured_ceilings(device).items():
            print(json.dumps({k: v}))


def measured_ceilings(device, nbytes=1 << 30):
    """Streaming ceilings of this chip measured with the csrc/probe.hip kernels (1 GiB,
    beyond the 256 MiB Infinity Cache) and torch's copy, in GB/s."""
    import ctypes

    from accdfl_amd import _lib

    so = ctypes.CDLL(_lib.build_probe())
    so.dlp_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                            ctypes.c_void_p]
    so.dlp_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=device).normal_()
    b = torch.empty_like(a)
    sink = torch.zeros(1024, dtype=torch.int32, device=device)
    sp = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    res = {}
    for ch in (1, 4, 8):
        for nt in (0, 1):
            _, ev = time_kernel(lambda: so.dlp_read(a.data_ptr(), nbytes, sink.data_ptr(), ch, nt, sp()), 30, 3, 1, settle_s=0.02)
            res["read_ch%d_nt%d" % (ch, nt)] = round(nbytes / (ev / 30) / 1e9, 1)
    for nt in (0, 1):
        _, ev = time_kernel(lambda: so.dlp_copy(a.data_ptr(), b.data_ptr(), nbytes, nt, sp()), 30, 3, 1, settle_s=0.02)
        res["copy_nt%d" % nt] = round(2 * nbytes / (ev / 30) / 1e9, 1)
    _, ev = time_kernel(lambda: b.copy_(a), 30, 3, 1, settle_s=0.02)
    res["torch_copy"] = round(2 * nbytes / (ev / 30) / 1e9, 1)
    del a, b
    # the FedAvg access pattern without arithmetic: 8 streams of 100 MB (+ 1 output stream)
    each = 100_000_000
    srcs = torch.empty((8, each // 4), dtype=torch.float32, device=device).normal_()
    dst = torch.empty(each // 4, dtype=torch.float32, device=device)
    arr = (ctypes.c_void_p * 8)(*[srcs[k].data_ptr() for k in range(8)])
    so.dlp_mread8.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_int, ctypes.c_void_p]
    for ch in (1, 2, 4):
        for wr in (0, 1, 2):
            _, ev = time_kernel(lambda: so.dlp_mread8(arr, each, dst.data_ptr(), sink.data_ptr(), ch, wr, sp()),
                                30, 3, 1)
            res["mread8_ch%d_write%s" % (ch, ("0", "1", "1_sc1")[wr])] = round((8 + min(wr, 1)) * each /
                                                                                (ev / 30) / 1e9, 1)
        _, ev = time_kernel(lambda: so.dlp_mread8(arr, each, srcs[0].data_ptr(), sink.data_ptr(), ch, 1, sp()),
                            30, 3, 1)
        res["mread8_ch%d_write_inplace" % ch] = round(9 * each / (ev / 30) / 1e9, 1)
    so.dlp_policy8.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    for rnd in range(3):
        for pol, name in enumerate(("nt", "sc1", "sc0sc1", "sc0sc1nt", "sc1nt")):
            _, ev = time_kernel(lambda: so.dlp_policy8(arr, each, dst.data_ptr(), pol, sp()), 30, 3, 1, settle_s=0.02)
            res["policy8_%s_r%d" % (name, rnd)] = round(9 * each / (ev / 30) / 1e9, 1)
    del srcs
    # tile-interleaved peer layout ([tiles][8 (+1 out)][T]) — one contiguous region per workgroup
    slab9 = torch.empty(9 * each // 4, dtype=torch.float32, device=device).normal_()
    so.dlp_tiled8.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                              ctypes.c_void_p]
    for ch in (1, 4, 16):
        for slot in (0, 1):
            _, ev = time_kernel(lambda: so.dlp_tiled8(slab9.data_ptr(), each, dst.data_ptr(), ch, slot, sp()),
                                30, 3, 1)
            res["tiled8_ch%d_outslot%d" % (ch, slot)] = round(9 * each / (ev / 30) / 1e9, 1)
    return res


def main():
    args = parse()
    global SETTLE_S
    SETTLE_S = args.settle_ms / 1e3
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))  # nothing has touched a GPU in this process
    rank, world, device, cpu_group = setup_dist(args)
    if args.dry_run:
        dry_run(args, rank, world, cpu_group)
        return
    from accdfl_amd import _lib
    from accdfl_amd.core import wsum
    from accdfl_amd.core.host_memory import bind_to_gpu_node

    _lib.lib()  # fail loudly here if the HIP library is missing
    # one process per GPU, bound to the GPU's NUMA node before any host buffer is allocated: the
    # host-inclusive legs then pack and DMA node-local memory (configs[4] CPU modules: 159-177 ms
    # unbound, 111-121 bound, profiles/r02zb)
    numa_node = None if args.no_numa_bind else bind_to_gpu_node(device)
    if args.sweep:
        sweep(args, device)
        return
    if args.host_breakdown:
        print(json.dumps(host_breakdown(args.peers, args.params, device)))
        return
    if args.host_configs_only:
        print(json.dumps(dict(config="north star 8 x 25 M f32 (one tensor per peer)",
                              **host_inclusive(args.peers, args.params))), flush=True)
        print(json.dumps(dict(config="GNLeNet small rounds", numa_node_bound=numa_node, **host_inclusive_small())),
              flush=True)
        for name, row in host_inclusive_configs().items():
            print(json.dumps(dict(config=name, **row)), flush=True)
        return
    if args.device_configs_only:
        for name, row in device_module_configs(device).items():
            print(json.dumps(dict(config=name, **row)), flush=True)
        return
    if args.configs_only:
        for name, row in baseline_configs(device).items():
            print(json.dumps(dict(config=name, **row)))
        return
    dt = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}[args.dtype]
    es = 4 if args.dtype == "f32" else 2
    n, p = args.peers, args.params
    # this rank's bucket of every peer, resident in HBM as PeerSlab stages it: the
    # tile-interleaved slab (core/peer_slab.py; --layout rows: one buffer per peer)
    w = [float(x) for x in np.random.default_rng(0).dirichlet(np.ones(n))]
    cfg = None
    if args.variant or args.chunks or args.grid or args.block:
        cfg = _lib.LaunchCfg(args.variant, args.chunks, args.grid, args.block)
    code = wsum.dtype_code(dt)
    result = {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "launch": dict(launch_info(world), numa_node_bound=numa_node)}
    legs = Legs(rank, world, cpu_group, args.leg_timeout, result)
    legs.arm("headline (setup)")
    inp = SlabInput(n, p, dt, device, 1000 + 97 * rank, w, layout="rows" if cfg is not None else args.layout)
    if cfg is not None:
        ptrs = [inp.buf[k].data_ptr() for k in range(n)]

        def step():
            _lib.wsum_ptrs(code, ptrs, w, p, inp.out.data_ptr(), torch.cuda.current_stream().cuda_stream, cfg)
    else:
        def step():
            inp.launch(torch.cuda.current_stream().cuda_stream)

    log("headline: %d peers x %d %s, %d ranks" % (n, p, args.dtype, world))
    legs.arm("headline")
    wall, ev = time_kernel(step, args.steps, args.warmup, world)
    legs.disarm()
    bytes_step = (n + 1) * p * es
    ms_per_step = wall / args.steps * 1e3
    value = world * bytes_step / (wall / args.steps) / 1e9
    kern_s = ev / args.steps
    achieved = bytes_step / kern_s / 1e9
    traffic = None
    if os.path.exists(PMC_FILE):
        try:
            pm = json.load(open(PMC_FILE))
            if (pm.get("workload") == "ns" and pm.get("peers") == n and pm.get("params") == p
                    and pm.get("layout", "rows") == inp.layout and cfg is None):
                traffic = pm.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    result.update({
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (per-peer seeded normal(0, 0.05), Dirichlet(1) weights), inputs resident in HBM",
        "config": {
            "workload": "north-star FedAvg reduce: %d peers x %d %s params per GPU (one parameter bucket per "
                        "GPU of a %d-GPU bucket-sharded model)" % (n, p, args.dtype, world),
            "n_peers": n,
            "params_per_gpu": p,
            "global_params": p * world,
            "parallelism": "bucket-sharded x%d (no data-path collective)" % world,
            "hbm_layout": ("PeerSlab tile-interleaved slab [n_tiles][%d peers][%d-element tiles]" % (n, inp.tile)
                           if inp.layout == "slab" else "one buffer per peer"),
        },
        "launch": dict(launch_info(world), numa_node_bound=numa_node),
        "roofline": {
            "bound": "hbm",
            "kernel": inp.kernel if cfg is None else "forced launch cfg %s" % (tuple(args_cfg(args)),),
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "bytes_per_launch": bytes_step,
            "us_per_launch": round(kern_s * 1e6, 2),
        },
    })
    parity = result["parity"] = {}
    if world > 1:
        row = legs.run("headline_parity", leg_headline_parity, inp, n, p, dt, w, rank, world, device)
        parity["headline (all-gathered buckets vs one-GPU reduce of the whole model)"] = row.get("parity_ok")
        result["headline_parity"] = row
    head_out = inp.out[:p].clone()
    headline_host = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.dtype == "f32" and cfg is None:
        # the headline's peers and output on the host, for the oracle check in the cpu_baseline leg
        # (after the timed region; the peers are regenerated exactly as SlabInput made them)
        pitch = max(128, (p + 127) // 128 * 128)
        rows = make_slab(n, pitch, dt, device, 1000 + 97 * rank)
        headline_host = ([rows[k, :p].cpu() for k in range(n)], head_out.cpu())
        del rows
    del inp
    torch.cuda.empty_cache()
    if cfg is None and args.layout == "slab":
        def separate(L):
            # the same peers as separate buffers (what FedAvg.aggregate on device modules reduces)
            rows = SlabInput(n, p, dt, device, 1000 + 97 * rank, w, layout="rows")
            L.go()
            _, ev_r = time_kernel(lambda: rows.launch(torch.cuda.current_stream().cuda_stream), args.steps,
                                  args.warmup, world)
            L.settled()
            row = {"kernel": rows.kernel, "us_per_launch": round(ev_r / args.steps * 1e6, 2),
                   "GB/s": round(bytes_step / (ev_r / args.steps) / 1e9, 1),
                   "parity_ok": same_bits(rows.out[:p], head_out),
                   "check": "same peers, row-major kernel == the headline's tiled-slab kernel, bit for bit"}
            del rows
            torch.cuda.empty_cache()
            return row
        result["separate_buffers"] = legs.run("separate_buffers", separate)
        parity["separate_buffers == headline"] = result["separate_buffers"].get("parity_ok")
    del head_out
    if not args.no_strong and args.dtype == "f32" and (n, p) == (NS_PEERS, NS_PARAMS):
        lines = {}
        for name in STRONG:
            lines[name] = legs.run("strong: " + name, strong_line, name, rank, world, device, args.strong_steps, 3)
            if world > 1:
                parity["strong: " + name] = lines[name].get("parity_ok")
        result["strong_scaling"] = {"scaling": "strong", "lines": lines}
        # BASELINE's fixed-model multi-GPU configs as top-level figures: the north star
        # split N ways, configs[3'] (64 ResNet-8 models; configs[3] names 4 GPUs) and configs[4] (128
        # ResNet-34 bf16; 8 GPUs), each against the same model on one GPU of this run
        strong = result["strong_headline"] = {"scaling": "strong", "n_gpus": world}
        for key, name in (("north_star", "north star, 8 peers x 25 M f32"),
                          ("configs3_resnet8", "configs[3'] CIFAR-10 ResNet-8, 64 peers"),
                          ("configs4_resnet34_bf16", "configs[4] google_speech ResNet-34, 128 peers, bf16")):
            ln = lines.get(name) or {}
            strong[key] = {k: ln.get(k) for k in ("value", "ms_per_step", "one_gpu_value", "speedup_vs_one_gpu",
                                                  "efficiency", "allgather_ms", "with_allgather_value",
                                                  "speedup_with_allgather", "parity_ok", "skipped", "error")
                           if k in ln}
            if world == 1 and "value" in ln:
                strong[key].update(one_gpu_value=ln["value"], speedup_vs_one_gpu=1.0, efficiency=1.0)
    if world > 1 and not args.no_collectives:
        coll_p = args.coll_params or (p if dist.get_backend() == "nccl" else min(p, 1 << 21))
        coll = result["collectives"] = {}
        coll["allgather"] = legs.run("allgather", leg_allgather, coll_p, dt, es, world, rank, device)
        for exact, key in ((True, "peer_sharded_exact"), (False, "peer_sharded_reduce_scatter")):
            coll[key] = legs.run(key, leg_peer_sharded, exact, n, coll_p, dt, world, rank, device, w)
        if args.dtype == "f32":
            coll["xgmi_sharded"] = legs.run("xgmi_sharded", leg_xgmi_sharded, n, p, world, rank, device, w)
        for key, row in coll.items():
            parity["collectives: " + key] = row.get("parity_ok")
    if world > 1 and not args.no_host_inclusive and args.dtype == "f32":
        # rank 0 alone drives GPUs 0..G-1 from one process (the reference's CPU-module call
        # sites); the other ranks wait on the CPU (gloo), so no RCCL kernel sits on a GPU
        def sharded_host(L):
            L.go()
            return host_inclusive_sharded(n, p, world) if rank == 0 else {}
        result["host_inclusive_sharded"] = legs.run("host_inclusive_sharded", sharded_host)
        parity["host_inclusive_sharded"] = result["host_inclusive_sharded"].get("parity_ok")
    if rank == 0 and world == 1:
        if not args.no_small:
            result["baseline_configs"] = legs.run("baseline_configs", lambda L: baseline_configs(device))
            result["device_module_configs"] = legs.run("device_module_configs",
                                                       lambda L: device_module_configs(device))
            parity["device round of reference module trees == ParameterList layout"] = \
                result["device_module_configs"].get(TREE_CONFIG, {}).get("parity_ok")
        if not args.no_host_inclusive and args.dtype == "f32":
            result["host_inclusive"] = legs.run("host_inclusive", lambda L: host_inclusive(n, p))
            result["wire_ingress"] = legs.run("wire_ingress", lambda L: wire_ingress(p, device))
            result["host_inclusive_small"] = legs.run("host_inclusive_small", lambda L: host_inclusive_small())
            result["host_inclusive_configs"] = legs.run("host_inclusive_configs", lambda L: host_inclusive_configs())
            for cname, crow in result["host_inclusive_configs"].items():
                if isinstance(crow, dict) and "staged_parity_ok" in crow:
                    parity["staged on arrival == FedAvg.aggregate: " + cname] = crow["staged_parity_ok"]

            def dfl(L):
                msgs = dfl_messages(n, p)
                return dfl_round(msgs, p, device)
            result["dfl_round"] = legs.run("dfl_round", dfl)
            result["dfl_round_layout"] = legs.run(
                "dfl_round_layout", lambda L: dfl_round_layout("google_speech_resnet34", 16, torch.bfloat16, device))
            parity["dfl_round_layout (wire ingress of 110 tensors == device FedAvg)"] = \
                result["dfl_round_layout"].get("parity_ok")
        if not args.no_cpu_baseline and args.dtype == "f32":
            result["cpu_baseline"] = legs.run("cpu_baseline",
                                              lambda L: cpu_baseline_all(args, result, n, p, headline_host),
                                              timeout_s=max(args.leg_timeout, 600))
            headline_host = None
            hp = result["cpu_baseline"].get("headline_oracle_parity")
            if hp is not None:
                parity["headline == reference op sequence (oracle port, every element)"] = hp.get("parity_ok")
                result["headline_oracle_parity"] = hp
    parity = {k: v for k, v in parity.items() if v is not None}
    result["parity"] = parity
    result["parity_ok"] = all(parity.values()) if parity else None
    result["legs_failed"] = legs.failed
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
