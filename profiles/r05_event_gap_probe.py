"""Round 5: does an event recorded on the stream after every reduce cost GPU time between kernels?

The table reduce's ring (core/wsum.py _TableRing) records a torch event after every call so a slot is
reused only once the stream has passed it; the kernel trace of back-to-back table reduces shows ~6 us
between consecutive kernels against ~2 us for the headline's prepared launches, which record nothing.
This times the headline reduce (8 x 25 M fp32, prepared launch) back to back with no event, with a
fresh torch event recorded after each launch, and with one event re-recorded after each launch."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

import bench  # noqa: E402


def main():
    device = torch.device("cuda", 0)
    n, p = 8, 25_000_000
    w = [float(x) for x in np.random.default_rng(0).dirichlet(np.ones(n))]
    inp = bench.SlabInput(n, p, torch.float32, device, 1000, w)
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    one = torch.cuda.Event()

    def plain():
        inp.launch(sp)

    def fresh_event():
        inp.launch(sp)
        torch.cuda.Event().record(s)

    def same_event():
        inp.launch(sp)
        one.record(s)

    for name, fn in (("no_event", plain), ("fresh_event", fresh_event), ("same_event", same_event),
                     ("no_event_again", plain)):
        evs = [bench.time_kernel(fn, 100, 5, 1, settle_s=0.05)[1] for _ in range(3)]
        print(json.dumps({"variant": name, "us_per_launch": [round(e / 100 * 1e6, 2) for e in evs]}), flush=True)


if __name__ == "__main__":
    main()
