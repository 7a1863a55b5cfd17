"""Round 5: what a peer's H2D into the tile-interleaved PeerSlab costs, host side and copy-engine side.

The DFL round's phase split (bench.py dfl_round, profiles/r05j/bench.log) spends 0.79 ms of host time per
100 MB peer issuing its dla_slab_stage copy and moves the peers at 52 GB/s against the link's ~57.  This
times, for one 100 MB fp32 peer in a page-locked buffer (an ingress buffer), each way of landing it in
row k of an 8-row slab of 32 KiB tiles — the host time of the issuing call and the copy's time by events:
  2d      dla_slab_stage: one hipMemcpy2DAsync (rows = tiles, destination pitch = 8 tiles)
  linear  a plain hipMemcpyAsync of the 100 MB into a contiguous device buffer (the link's rate)
  lin+2d  the linear H2D into a contiguous device chunk, then dla_slab_stage device -> slab (D2D 2D)
Every variant's slab row is checked against the source."""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

from accdfl_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n_rows, p = 8, 25_000_000
    tile = _lib.slab_tile_elems(_lib.DLA_F32, n_rows, p)
    n_t = -(-p // tile)
    slab = torch.zeros((n_t, n_rows, tile), dtype=torch.float32, device=dev)
    src = torch.empty(p, dtype=torch.float32, pin_memory=True)
    src.copy_(torch.randn(p, generator=torch.Generator().manual_seed(3)))
    lin = torch.empty(p, dtype=torch.float32, device=dev)
    s = torch.cuda.Stream(dev)
    sp = int(s.cuda_stream)

    def check(row):
        got = slab[:, row, :].reshape(-1)[:p].cpu()
        return bool(torch.equal(got, src))

    def v_2d(row):
        _lib.slab_stage(_lib.DLA_F32, slab.data_ptr(), tile, n_rows, n_t, row, 0, src.data_ptr(), p, sp)

    def v_linear(row):
        with torch.cuda.stream(s):
            lin.copy_(src, non_blocking=True)

    def v_lin2d(row):
        with torch.cuda.stream(s):
            lin.copy_(src, non_blocking=True)
        _lib.slab_stage(_lib.DLA_F32, slab.data_ptr(), tile, n_rows, n_t, row, 0, lin.data_ptr(), p, sp)

    out = {"tile_bytes": tile * 4, "peer_MB": p * 4 / 1e6}
    for name, fn in (("2d", v_2d), ("linear", v_linear), ("lin+2d", v_lin2d), ("2d_again", v_2d)):
        host_ms, dev_ms = [], []
        for rep in range(8):
            row = rep % n_rows
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            t0 = time.perf_counter()
            fn(row)
            host_ms.append((time.perf_counter() - t0) * 1e3)
            e1.record(s)
            e1.synchronize()
            dev_ms.append(e0.elapsed_time(e1))
        ok = check(row) if name != "linear" else bool(torch.equal(lin.cpu(), src))
        out[name] = {"host_issue_ms": round(statistics.median(host_ms), 3), "copy_ms": round(statistics.median(dev_ms), 3),
                     "GB/s": round(p * 4 / statistics.median(dev_ms) / 1e6, 1), "bit_exact": ok}
        print(json.dumps({name: out[name]}), flush=True)
    # a burst: every row issued back to back from its own page-locked buffer with no wait in between
    # (the DFL round's pattern: the next peer is issued while the previous one's copy still runs) —
    # does an issuing call return at once, or wait for the copy before it?
    bufs = [torch.empty(p, dtype=torch.float32, pin_memory=True) for _ in range(n_rows)]
    for b in bufs:
        b.copy_(src)
    for name in ("burst_2d", "burst_linear"):
        lins = [torch.empty(p, dtype=torch.float32, device=dev) for _ in range(2)] if name == "burst_linear" else None
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        calls = []
        t0 = time.perf_counter()
        for row in range(n_rows):
            tc = time.perf_counter()
            if name == "burst_2d":
                _lib.slab_stage(_lib.DLA_F32, slab.data_ptr(), tile, n_rows, n_t, row, 0, bufs[row].data_ptr(), p, sp)
            else:
                with torch.cuda.stream(s):
                    lins[row & 1].copy_(bufs[row], non_blocking=True)
            calls.append(round((time.perf_counter() - tc) * 1e3, 3))
        t_issue = (time.perf_counter() - t0) * 1e3
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        ok = all(torch.equal(slab[:, r, :].reshape(-1)[:p].cpu(), src) for r in range(n_rows)) if name == "burst_2d" else None
        out[name] = {"issue_ms_per_call": calls, "issue_total_ms": round(t_issue, 3), "copies_ms": round(ms, 3),
                     "GB/s": round(n_rows * p * 4 / ms / 1e6, 1), "bit_exact": ok}
        print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
