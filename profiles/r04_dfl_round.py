"""r04: bench.py's dfl_round leg alone (8 EVA-block messages of a 25 M fp32 model), with its phase split,
on the GPU's NUMA node as bench.py binds it; ``--runs R`` repeats the whole leg R times in one process.
Usage on the GPU box: python profiles/r04_dfl_round.py [--runs 3] -> one JSON line per run."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402

from accdfl_amd.core.host_memory import bind_to_gpu_node  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--runs", type=int, default=3)
args = ap.parse_args()
node = bind_to_gpu_node()
msgs = bench.dfl_messages(8, 25_000_000)
for r in range(args.runs):
    row = bench.dfl_round(msgs, 25_000_000, torch.device("cuda", 0), reps=5)
    row["numa_node_bound"] = node
    row["run"] = r
    print(json.dumps(row), flush=True)
