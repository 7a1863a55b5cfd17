"""Round 5: the occupancy cap on the strong-split buckets.  The cap rule applies from
256 MiB of input; the north star's 4- and 8-way buckets (8 x 6.25 M / 3.125 M f32: 200 / 100 MB) run
uncapped and read 0.80 / 0.74 of peak against 0.89 for the whole model (profiles/r05o).  Times those
buckets (and the 2-way one, capped by the rule) under the cap the tuning build takes from
DLA_VEC_WGS_PER_CU (run once per value; unset = the product rule), rotated input copies as strong_line.
Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "decentralized-learning_amd"))

import bench  # noqa: E402
from r05_strong_share_probe import share_s  # noqa: E402

SHAPES = [(8, 12_500_032, "f32"), (8, 6_250_048, "f32"), (8, 3_125_056, "f32"), (64, 1_233_088, "f32"),
          (64, 616_576, "f32")]


def main():
    device = torch.device("cuda", 0)
    row = {"DLA_VEC_WGS_PER_CU": os.environ.get("DLA_VEC_WGS_PER_CU", "rule")}
    for n, m, dts in SHAPES:
        dt = torch.float32 if dts == "f32" else torch.bfloat16
        w = [float(x) for x in np.random.default_rng(0).dirichlet(np.ones(n))]
        t, t_ev, _ = share_s(n, m, dt, 4 if dts == "f32" else 2, device, w)
        row["%dx%d" % (n, m)] = [round(t * 1e6, 2), round(t_ev * 1e6, 2)]
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
