"""Round 5: where the DFL round's per-peer host time goes (bench.py dfl_round: decode + gather 1.05 ms and
"stage issue" 0.79 ms per 100 MB peer, while the 2D copy call itself returns in 5 us,
profiles/r05l/stage.log).  Runs bench.py's dfl_round ingress loop (8 messages of a 25 M fp32 model from
60 000-byte EVA blocks into a DeviceModelManager) under cProfile and prints the top functions by
cumulative and by own time, plus the loop's wall time with and without the phase events."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

import bench  # noqa: E402


def main():
    from types import SimpleNamespace

    from torch import nn

    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager

    dev = torch.device("cuda", 0)
    if "--bind" in sys.argv:  # as bench.py does before its legs (host_memory.bind_to_gpu_node)
        from accdfl_amd.core.host_memory import bind_to_gpu_node

        print("bound to NUMA node", bind_to_gpu_node(dev), "affinity", len(os.sched_getaffinity(0)), flush=True)
    n, p = 8, 25_000_000
    msgs = bench.dfl_messages(n, p)
    template = nn.Module()
    template.w = nn.Parameter(torch.zeros(p))
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0,
                            capacity=n, template=template, device=dev)

    def loop(phases):
        mm.reset_incoming_trained_models()
        if phases:
            mm.start_phases()
        t0 = time.perf_counter()
        for k, (blocks, ml) in enumerate(msgs):
            head, _ = wire.split_blocks(blocks, ml)
            mm.process_incoming_serialized(b"peer%d" % k, head)
        t1 = time.perf_counter()
        mm.slab.copy_stream.synchronize()
        t2 = time.perf_counter()
        mm.phases = None
        return (t1 - t0) * 1e3, (t2 - t0) * 1e3

    for _ in range(2):
        loop(False)
    for phases in (False, True, False, True):
        a, b = loop(phases)
        print("phases=%s loop %.2f ms, complete %.2f ms" % (phases, a, b), flush=True)
    if "--bench-round" in sys.argv:  # bench.py's own dfl_round (3 reps after one warm-up), phases included
        import json

        print(json.dumps(bench.dfl_round(msgs, p, dev)), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    loop(False)
    pr.disable()
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(28)
        print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
