"""r04: where the DFL aggregator round's ingress goes.  bench.py's dfl_round (8 EVA-block
messages of a 25 M fp32 model -> DeviceModelManager -> average -> bytes), five rounds, with EVERY peer's
phases kept (not medians): the wire split, the decode + gather into the page-locked ingress buffer (and the
native gather alone), the stage call, and the copy stream's own time for each peer's H2D + tile scatter
(HIP events), plus the wait for the copy stream after the loop.
Usage on the GPU box: python profiles/r04_dfl_phases.py -> JSON lines."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402

from accdfl_amd import _lib  # noqa: E402
from accdfl_amd.core import wire  # noqa: E402
from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod  # noqa: E402
from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402
from accdfl_amd.core.model_manager import DeviceModelManager  # noqa: E402


def main():
    node = bind_to_gpu_node()
    dev = torch.device("cuda", 0)
    p, n = 25_000_000, 8
    msgs = bench.dfl_messages(n, p)
    print(json.dumps({"numa_node_bound": node, "affinity_cpus": len(os.sched_getaffinity(0))}), flush=True)
    from types import SimpleNamespace
    from torch import nn

    template = nn.Module()
    template.w = nn.Parameter(torch.zeros(p))
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0,
                            capacity=n, template=template, device=dev)
    gather_t = []
    orig_copy = _lib.host_copy_batch

    def timed_copy(*a, **kw):
        t0 = time.perf_counter()
        try:
            return orig_copy(*a, **kw)
        finally:
            gather_t.append(time.perf_counter() - t0)
    _lib.host_copy_batch = timed_copy
    try:
        for rnd in range(6):
            mm.reset_incoming_trained_models()
            torch.cuda.synchronize()
            rows = []
            evs = []
            t_loop = time.perf_counter()
            for k, (blocks, ml) in enumerate(msgs):
                t0 = time.perf_counter()
                head, _ = wire.split_blocks(blocks, ml)
                t1 = time.perf_counter()
                g0 = len(gather_t)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                cs = mm.slab.copy_stream if mm.slab is not None else None
                if cs is not None:
                    e0.record(cs)
                mm.process_incoming_serialized(b"peer%d" % k, head)
                t2 = time.perf_counter()
                e1.record(mm.slab.copy_stream)
                evs.append((e0 if cs is not None else None, e1))
                rows.append({"split": t1 - t0, "decode_gather_stage": t2 - t1,
                             "native_gather": sum(gather_t[g0:])})
            t_end = time.perf_counter()
            mm.slab.copy_stream.synchronize()
            t_wait = time.perf_counter()
            out = mm.aggregate_serialized()
            t_agg = time.perf_counter()
            del out
            copy_ms = [round(a.elapsed_time(b), 3) if a is not None else None for a, b in evs]
            gaps = []
            for i in range(1, len(evs)):  # idle of the copy stream between peers
                gaps.append(round(evs[i - 1][1].elapsed_time(evs[i][0]), 3) if evs[i][0] is not None else None)
            print(json.dumps({
                "round": rnd, "loop_ms": round((t_end - t_loop) * 1e3, 2),
                "wait_copy_stream_ms": round((t_wait - t_end) * 1e3, 2),
                "aggregate_serialized_ms": round((t_agg - t_wait) * 1e3, 2),
                "per_peer_split_ms": [round(r["split"] * 1e3, 3) for r in rows],
                "per_peer_decode_gather_stage_ms": [round(r["decode_gather_stage"] * 1e3, 3) for r in rows],
                "per_peer_native_gather_ms": [round(r["native_gather"] * 1e3, 3) for r in rows],
                "per_peer_copy_stream_ms": copy_ms, "copy_stream_gap_ms": gaps}), flush=True)
    finally:
        _lib.host_copy_batch = orig_copy


if __name__ == "__main__":
    main()
