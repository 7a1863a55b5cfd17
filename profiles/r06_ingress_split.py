"""Round 6: where the native wire ingress of a many-tensor peer spends its host time — 16 google_speech
ResNet-34 bf16 payloads (110 parameters, 108 buffers, 42.7 MB each) as 60 000-byte EVA blocks, each step
of DeviceModelManager.process_incoming_serialized timed alone, medians over the peers of 3 rounds:
  scan       — wire.scan_state_dict (block table + the native pickle scan);
  row_layout — StateDictScan.row_layout (offsets of the parameters back to back);
  gather     — StateDictScan.gather (one batched memcpy into the page-locked ingress buffer);
  stage      — PeerSlab.stage_flat (the call that enqueues the row's copy);
plus the whole process_incoming_serialized per peer and the copy stream's time per peer."""
import json
import os
import pickle
import statistics
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "decentralized-learning_amd")]
import bench  # noqa: E402


def main():
    from accdfl_amd.core import wire
    from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod
    from accdfl_amd.core.model_manager import DeviceModelManager

    dev = torch.device("cuda", 0)
    if "--numa-bind" in sys.argv:  # as bench.py does per rank: the gather's threads near the GPU's PCIe root
        from accdfl_amd.core.host_memory import bind_to_gpu_node

        bind_to_gpu_node(dev)
    n = 16
    models, p = bench._layout_models("google_speech_resnet34", n, torch.bfloat16, pinned=False, seed=4200)
    view = pickle.dumps({"peer%d" % j: j for j in range(16)})
    msgs = []
    for m in models:
        mb = wire.serialize_model(m)
        msgs.append((wire.payload_blocks(mb + view, bench.EVA_BLOCK), len(mb)))
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0,
                            capacity=n, template=models[0], device=dev)
    names, shapes = mm._row_spec()
    split = {k: [] for k in ("scan", "row_layout", "gather", "stage", "whole")}
    for rnd in range(4):
        mm.reset_incoming_trained_models()
        for k, (blocks, ml) in enumerate(msgs):
            head, _ = wire.split_blocks(blocks, ml)
            t0 = time.perf_counter()
            mm.process_incoming_serialized(b"p%d" % k, head)
            t1 = time.perf_counter()
            if rnd:
                split["whole"].append(t1 - t0)
        mm.slab.copy_stream.synchronize()
    # the same steps one by one (into a page-locked buffer and a slab row of their own)
    buf = torch.empty(60 << 20, dtype=torch.uint8, pin_memory=True)
    slab = mm.slab
    for rnd in range(3):
        slab.reset()
        for k, (blocks, ml) in enumerate(msgs):
            head, _ = wire.split_blocks(blocks, ml)
            t0 = time.perf_counter()
            sc = wire.scan_state_dict(head)
            t1 = time.perf_counter()
            offsets, total, row = sc.row_layout(names, torch.bfloat16, shapes)
            t2 = time.perf_counter()
            sc.gather(buf[:total], offsets)
            t3 = time.perf_counter()
            slab.stage_flat(buf[:row].view(torch.bfloat16))
            t4 = time.perf_counter()
            slab.copy_stream.synchronize()
            for key, dt in (("scan", t1 - t0), ("row_layout", t2 - t1), ("gather", t3 - t2), ("stage", t4 - t3)):
                split[key].append(dt)
    out = {k: round(statistics.median(v) * 1e3, 4) for k, v in split.items()}
    out["peer_MB"] = round(len(wire.split_blocks(msgs[0][0], msgs[0][1])[0]) and msgs[0][1] / 1e6, 2)
    out["gather_GBps"] = round(msgs[0][1] / (out["gather"] / 1e3) / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
