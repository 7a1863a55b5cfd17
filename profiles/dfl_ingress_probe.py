"""r02: where one peer's EVA-block ingress (25 M fp32, 60 000-byte blocks) spends its time on
the GPU box: split, decode + gather into a page-locked buffer (per DLA_COPY_THREADS), the
batched gather alone, the PeerSlab stage (H2D + tile scatter)."""
import json
import os
import statistics
import sys
import time

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))
from accdfl_amd import _lib  # noqa: E402
from accdfl_amd.core import wire  # noqa: E402
from accdfl_amd.core.peer_slab import PeerSlab  # noqa: E402


def med(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e3, 2)


def main():
    p = 25_000_000
    m = nn.Module()
    m.w = nn.Parameter(torch.randn(p) * 0.05)
    data = wire.serialize_model(m)
    blocks = wire.payload_blocks(data, 60_000)
    pinned = torch.empty(len(data) + 4096, dtype=torch.uint8, pin_memory=True)
    pageable = torch.empty(len(data) + 4096, dtype=torch.uint8)
    pageable.fill_(0)
    res = {"blocks": len(blocks)}
    res["split_ms"] = med(lambda: wire.split_blocks(blocks, len(data)))
    head, _ = wire.split_blocks(blocks, len(data))
    res["decode_gather_pinned_ms"] = med(lambda: wire.loads_state_dict(head, copy=False, alloc=lambda n: pinned[:n]))
    addrs = [wire._block_address(b) for b in blocks]
    sizes = [len(b) for b in blocks]
    offs, o = [], 0
    for s in sizes:
        offs.append(o)
        o += s
    for name, buf in (("pinned", pinned), ("pageable", pageable)):
        base = buf.data_ptr()
        res["host_copy_batch_%s_ms" % name] = med(lambda: _lib.host_copy_batch([base + x for x in offs], addrs, sizes))
    res["one_memcpy_100MB_pinned_ms"] = med(lambda: pinned[: p * 4].copy_(m.w.detach().view(torch.uint8)))
    slab = PeerSlab([(p,)], torch.float32, capacity=8)
    sd = wire.loads_state_dict(head, copy=False, alloc=lambda n: pinned[:n])

    def stage():
        slab.reset()
        slab.stage([sd["w"]])
        slab.copy_stream.synchronize()
    res["stage_from_pinned_ms"] = med(stage)
    sd2 = wire.loads_state_dict(data, copy=False)

    def stage2():
        slab.reset()
        slab.stage([sd2["w"]])
        slab.copy_stream.synchronize()
    res["stage_from_payload_bytes_ms"] = med(stage2)
    res["threads_env"] = os.environ.get("DLA_COPY_THREADS", "default 8")
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
