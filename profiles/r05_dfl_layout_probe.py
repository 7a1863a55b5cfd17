"""Round 5: where a many-tensor DFL round's ingress time goes (bench.py dfl_round_layout: 16 google_speech
ResNet-34 bf16 models through 60 000-byte EVA blocks took 194 ms, 3.5 GB/s, against 16 ms for the
one-tensor 800 MB round, profiles/r05ai).  Per-arrival phases (decode + gather, stage issue, copy-engine
busy time) and a cProfile of the ingress loop sorted by own time; also the decode alone from the joined
bytes and from the blocks."""
import cProfile
import io
import json
import os
import pickle
import pstats
import statistics
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

import bench  # noqa: E402
from accdfl_amd.core import wire  # noqa: E402
from accdfl_amd.core.gradient_aggregation import GradientAggregationMethod  # noqa: E402
from accdfl_amd.core.model_manager import DeviceModelManager  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    name = sys.argv[1] if len(sys.argv) > 1 else "google_speech_resnet34"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dt = torch.bfloat16 if name == "google_speech_resnet34" else torch.float32
    models, p = bench._layout_models(name, n, dt, pinned=False, seed=4200)
    view = pickle.dumps({"peer%d" % j: j for j in range(16)})
    msgs = []
    for m in models:
        mb = wire.serialize_model(m)
        msgs.append((wire.payload_blocks(mb + view, bench.EVA_BLOCK), len(mb), mb))
    mm = DeviceModelManager(None, SimpleNamespace(gradient_aggregation=GradientAggregationMethod.FEDAVG), 0,
                            capacity=n, template=models[0], device=dev)

    def loop(phases):
        mm.reset_incoming_trained_models()
        ph = mm.start_phases() if phases else None
        t0 = time.perf_counter()
        for k, (blocks, ml, _) in enumerate(msgs):
            head, _ = wire.split_blocks(blocks, ml)
            mm.process_incoming_serialized(b"peer%d" % k, head)
        t1 = time.perf_counter()
        mm.slab.copy_stream.synchronize()
        t2 = time.perf_counter()
        mm.phases = None
        out = {"loop_ms": round((t1 - t0) * 1e3, 2), "complete_ms": round((t2 - t0) * 1e3, 2)}
        if ph is not None:
            out["decode_gather_ms"] = round(sum(ph["decode_gather_ms"]), 2)
            out["stage_issue_ms"] = round(sum(ph["stage_issue_ms"]), 2)
            out["copy_busy_ms"] = round(sum(a.elapsed_time(b) for a, b in ph["copy_events"]), 2)
        return out

    loop(False)
    print(json.dumps({"config": name, "peers": n, "no_phases": [loop(False) for _ in range(3)]}), flush=True)
    print(json.dumps({"phases": [loop(True) for _ in range(3)]}), flush=True)
    # the decode alone: joined bytes (zero-copy views) and the block list gathered into a plain buffer
    blocks, ml, mb = msgs[0]
    head, _ = wire.split_blocks(blocks, ml)
    buf = torch.empty(len(mb) + 256 * 512, dtype=torch.uint8)

    def dec_blocks():
        off = [0]

        def alloc(nb):
            a = off[0]
            off[0] = a + (nb + 255) // 256 * 256
            return buf[a:a + nb]
        wire.loads_state_dict(head, copy=False, alloc=alloc)

    res = {}
    for nm, fn in (("bytes", lambda: wire.loads_state_dict(mb, copy=False)), ("blocks", dec_blocks),
                   ("pickle.loads (reference)", lambda: pickle.loads(mb))):
        fn()
        ts = []
        for _ in range(7):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        res[nm] = round(statistics.median(ts) * 1e3, 2)
    print(json.dumps({"decode_one_peer_ms": res, "payload_MB": round(len(mb) / 1e6, 2)}), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    loop(False)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
