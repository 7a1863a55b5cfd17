"""Seeded random calls of the C ABI's reduce entry points against the C oracle, bit for bit (NaN as
NaN): random dtypes, peer counts (one, two and three 128-peer passes), lengths, element offsets that
break 16-byte alignment, weights with IEEE specials, out aliasing peers[0].

* dla_wsum: peers and out at random element offsets of their own buffers;
* dla_wsum_multi_table / _acc: random tensor tables (some tensors misaligned, so the call splits them
  between the table kernel and per-tensor launches), and a round split in two calls whose second
  continues the first one's running sum;
* dla_slab_stage + dla_wsum_slab_tiled: random tile sizes and slab heights, every peer landed in 1-3
  pieces at arbitrary element offsets from page-locked host memory or from the device.

The reference (fedavg.py:20-25) is restated by oracle/fedavg_ref.c (c_oracle.py)."""
import os
import numpy as np
import pytest
import torch

from c_oracle import c_wsum
from oracle.fedavg_oracle import same_bits

pytestmark = pytest.mark.gpu

CODE = {"f32": 0, "bf16": 1, "f16": 2, "f64": 3}
TDT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}
IDT = {"f32": torch.int32, "bf16": torch.int16, "f16": torch.int16, "f64": torch.int64}
UDT = {"f32": np.uint32, "bf16": np.uint16, "f16": np.uint16, "f64": np.uint64}
ES = {"f32": 4, "bf16": 2, "f16": 2, "f64": 8}
_SPECIAL = [float("nan"), float("inf"), float("-inf"), -0.0, 1e-45, 3e38, 6.5e4, 1e-8]
_PEERS = [1, 2, 3, 5, 8, 9, 16, 17, 32, 33, 64, 100, 128, 129, 200, 256, 257]
# ACCDFL_AMD_FUZZ_SCALE=k runs k times the seeds (a long fuzz campaign; the suites keep the default)
N_CASES = 80 * int(os.environ.get("ACCDFL_AMD_FUZZ_SCALE", "1"))
_BUDGET = 12_000_000  # peer elements per case (host memory and oracle time)


def _host(rng, numel, dt, specials):
    x = rng.standard_normal(numel) * (10.0 ** rng.integers(-2, 3))
    if specials and numel:
        for i in rng.integers(0, numel, size=min(numel, 4)):
            x[i] = _SPECIAL[rng.integers(len(_SPECIAL))]
    with np.errstate(all="ignore"):
        return torch.from_numpy(x).to(TDT[dt])


def _bits(t: torch.Tensor, dt: str) -> np.ndarray:
    return t.detach().cpu().contiguous().view(IDT[dt]).numpy().view(UDT[dt])


def _weights(rng, n):
    w = [float(x) for x in (rng.dirichlet(np.ones(n)) if rng.integers(0, 2) else rng.standard_normal(n))]
    if rng.integers(0, 4) == 0:
        w[int(rng.integers(n))] = [0.0, float("nan"), float("inf"), 1e-40, -1e30][rng.integers(5)]
    return w


class _Placed:
    """A device buffer holding `host` at element offset `off` (so its pointer may be misaligned)."""

    def __init__(self, host: torch.Tensor, off: int):
        self.buf = torch.zeros(host.numel() + off + 8, dtype=host.dtype, device="cuda")
        self.buf[off:off + host.numel()].copy_(host)
        self.off, self.n = off, host.numel()

    @property
    def ptr(self) -> int:
        return self.buf.data_ptr() + self.off * self.buf.element_size()

    def view(self) -> torch.Tensor:
        return self.buf[self.off:self.off + self.n]


@pytest.mark.parametrize("seed", range(N_CASES))
def test_wsum_fuzz(seed):
    from accdfl_amd import _lib

    rng = np.random.default_rng(1000 + seed)
    dt = ["f32", "bf16", "f16", "f64"][rng.integers(4)]
    n = int(_PEERS[rng.integers(len(_PEERS))])
    numel = int([0, 1, 3, 8, 17, 255, 4096, 65_537, 300_001][rng.integers(9)])
    numel = min(numel, _BUDGET // n)
    specials = rng.integers(0, 3) == 0
    hosts = [_host(rng, numel, dt, specials) for _ in range(n)]
    peers = [_Placed(h, int(rng.integers(0, 8)) if rng.integers(0, 2) else 0) for h in hosts]
    w = _weights(rng, n)
    alias = rng.integers(0, 4) == 0
    out = peers[0] if alias else _Placed(torch.zeros(numel, dtype=TDT[dt]), int(rng.integers(0, 8)))
    want = c_wsum([_bits(h, dt) for h in hosts], w, dt)
    _lib.wsum_ptrs(CODE[dt], [p.ptr for p in peers], w, numel, out.ptr, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert same_bits(_bits(out.view(), dt), want, dt), \
        "seed %d: %s n=%d numel=%d alias=%s offsets=%s" % (seed, dt, n, numel, alias, [p.off for p in peers][:8])


def _table(n_tensors, n_peers):
    from accdfl_amd import _lib

    nb = _lib.wsum_multi_table_bytes(n_tensors, n_peers)
    return torch.empty(nb, dtype=torch.uint8, pin_memory=True), torch.empty(nb, dtype=torch.uint8, device="cuda")


@pytest.mark.parametrize("seed", range(N_CASES))
def test_multi_table_fuzz(seed):
    from accdfl_amd import _lib

    rng = np.random.default_rng(2000 + seed)
    dt = ["f32", "bf16", "f16", "f32", "bf16", "f64"][rng.integers(6)]
    n = int(_PEERS[rng.integers(len(_PEERS))])
    t = int(rng.integers(1, 25))
    numels = [int([0, 1, 2, 5, 64, 1000, 4099, 50_000, 131_072][rng.integers(9)]) for _ in range(t)]
    while n * sum(numels) > _BUDGET:
        numels[int(np.argmax(numels))] //= 4
    specials = rng.integers(0, 3) == 0
    misalign = rng.integers(0, 3) == 0
    hosts = [[_host(rng, m, dt, specials) for _ in range(n)] for m in numels]  # [tensor][peer]
    placed = [[_Placed(h, int(rng.integers(0, 8)) if misalign and rng.integers(0, 3) == 0 else 0) for h in row]
              for row in hosts]
    outs = [_Placed(torch.zeros(m, dtype=TDT[dt]), 0) for m in numels]
    w = _weights(rng, n)
    split = int(rng.integers(1, n)) if n > 1 and rng.integers(0, 2) else n
    sp = torch.cuda.current_stream().cuda_stream
    # first call: peers [0, split); second (acc): peers [split, n) folded into the running sum
    for lo, hi, acc in ((0, split, False), (split, n, True)):
        if lo >= hi:
            continue
        ptrs = [placed[i][k].ptr for i in range(t) for k in range(lo, hi)]
        th, td = _table(t, hi - lo)
        _lib.wsum_multi_table_ptrs(CODE[dt], ptrs, [o.ptr for o in outs], numels, w[lo:hi], th.data_ptr(),
                                   td.data_ptr(), sp, acc_in=acc)
        torch.cuda.synchronize()  # the table buffers are dropped after this call
    for i in range(t):
        want = c_wsum([_bits(h, dt) for h in hosts[i]], w, dt)
        assert same_bits(_bits(outs[i].view(), dt), want, dt), \
            "seed %d: %s n=%d split=%d tensor %d of %d numel=%d" % (seed, dt, n, split, i, t, numels[i])


@pytest.mark.parametrize("seed", range(N_CASES))
def test_slab_stage_and_tiled_reduce_fuzz(seed):
    from accdfl_amd import _lib

    rng = np.random.default_rng(3000 + seed)
    dt = ["f32", "bf16", "f16"][rng.integers(3)]
    es = ES[dt]
    rows = int(rng.integers(1, 21))
    n = int(rng.integers(1, rows + 1))
    numel = int([1, 7, 100, 4097, 33_333, 262_145, 1_000_003][rng.integers(7)])
    tile = (1 << int(rng.integers(4, 17))) // es  # 16 B .. 64 KiB
    n_tiles = -(-numel // tile) + int(rng.integers(0, 2))
    slab = torch.zeros((n_tiles, rows, tile), dtype=TDT[dt], device="cuda")
    specials = rng.integers(0, 3) == 0
    hosts = [_host(rng, numel, dt, specials) for _ in range(n)]
    sp = torch.cuda.current_stream().cuda_stream
    keep = []
    for k, h in enumerate(hosts):
        cuts = sorted({0, numel, *[int(c) for c in rng.integers(0, numel + 1, size=int(rng.integers(0, 3)))]})
        for a, b in zip(cuts[:-1], cuts[1:]):
            if rng.integers(0, 2):
                src = h[a:b].clone().pin_memory()
                ptr = src.data_ptr()
            else:
                src = _Placed(h[a:b], int(rng.integers(0, 4)))
                ptr = src.ptr
            keep.append(src)
            _lib.slab_stage(CODE[dt], slab.data_ptr(), tile, rows, n_tiles, k, a, ptr, b - a, sp)
    w = _weights(rng, n)
    out = torch.zeros(numel, dtype=TDT[dt], device="cuda")
    _lib.wsum_slab_tiled_ptr(CODE[dt], slab.data_ptr(), tile, rows, w, numel, out.data_ptr(), sp)
    torch.cuda.synchronize()
    staged = slab.permute(1, 0, 2).reshape(rows, -1)[:n, :numel].cpu()
    for k, h in enumerate(hosts):
        assert torch.equal(staged[k].view(IDT[dt]), h.view(IDT[dt])), "seed %d: row %d staged wrong" % (seed, k)
    want = c_wsum([_bits(h, dt) for h in hosts], w, dt)
    assert same_bits(_bits(out, dt), want, dt), \
        "seed %d: %s rows=%d n=%d numel=%d tile=%d" % (seed, dt, rows, n, numel, tile)


@pytest.mark.parametrize("seed", range(N_CASES // 2))
def test_mean_fuzz(seed):
    """dla_mean (scripts/distill.py:124-129's teacher-logit mean): (((+0 + p_0) + p_1) + ... ) / N in
    the storage type, correctly rounded division, peers and out at random offsets, out aliasing
    peers[0] across 128-peer passes; against numpy's sequential sum and IEEE division."""
    from accdfl_amd import _lib

    rng = np.random.default_rng(6000 + seed)
    dt = ["f32", "f64"][rng.integers(2)]
    n = int(_PEERS[rng.integers(len(_PEERS))])
    numel = min(int([1, 3, 64, 1000, 4097, 65_537, 300_001][rng.integers(7)]), _BUDGET // n)
    hosts = [_host(rng, numel, dt, rng.integers(0, 3) == 0) for _ in range(n)]
    peers = [_Placed(h, int(rng.integers(0, 4)) if rng.integers(0, 2) else 0) for h in hosts]
    alias = rng.integers(0, 3) == 0
    out = peers[0] if alias else _Placed(torch.zeros(numel, dtype=TDT[dt]), int(rng.integers(0, 4)))
    npdt = np.float32 if dt == "f32" else np.float64
    acc = np.zeros(numel, dtype=npdt)
    with np.errstate(all="ignore"):
        for h in hosts:
            acc = acc + h.numpy().astype(npdt)
        want = (acc / npdt(n)).view(UDT[dt])
    _lib.mean_ptrs(CODE[dt], [p.ptr for p in peers], numel, out.ptr, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert same_bits(_bits(out.view(), dt), want, dt), "seed %d: %s n=%d numel=%d alias=%s" % (seed, dt, n, numel,
                                                                                              alias)
