"""Round 5: per-channel and translation summaries of the table kernel against the
tiled kernel on the same bytes.  Reads rocprofv3 --pmc CSV passes (profiles/r05h_run.sh) and writes, per
(kernel, grid) and counter, the mean over dispatches of the counter summed over its dimension rows and —
for counters collected per TCC instance x XCC (TCC_EA0_RDREQ, TCC_BUSY: 16 x 8 = 128 channels) — the
spread over the channels: min / mean / max, max / mean and the coefficient of variation.  A pattern that
concentrates its concurrent reads on few channels shows max / mean well above 1.
Usage: python profiles/r05_pmc_channels.py OUT.json DIR [DIR ...]"""
import csv
import glob
import json
import os
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel)<([^>]*)>", name)
    return "%s<%s>" % (m.group(1), m.group(2)) if m else name[:100]


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    doc = {}
    for d in dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        rows = []
        for f in files:
            with open(f) as fh:
                rows.extend(csv.DictReader(fh))
        if not rows:
            doc[os.path.basename(d)] = {"error": "no counter_collection.csv"}
            continue
        cols = list(rows[0].keys())
        # (kernel key, counter) -> dispatch -> [values in row order (one per dimension instance)]
        acc = defaultdict(lambda: defaultdict(list))
        for r in rows:
            key = "%s grid=%s" % (short(r.get("Kernel_Name", "")), r.get("Grid_Size", r.get("Grid_Size_X", "?")))
            acc[(key, r.get("Counter_Name"))][r.get("Dispatch_Id")].append(float(r.get("Counter_Value") or 0))
        per = {}
        for (key, cname), disp in acc.items():
            if "wsum" not in key or len(disp) < 3:
                continue
            vals = list(disp.values())
            n_inst = max(len(v) for v in vals)
            row = {"dispatches": len(vals), "rows_per_dispatch": n_inst,
                   "mean_total": round(statistics.mean(sum(v) for v in vals), 1)}
            if n_inst > 1:
                per_inst = [statistics.mean(v[i] for v in vals if len(v) == n_inst) for i in range(n_inst)]
                mu = statistics.mean(per_inst)
                if mu > 0:
                    row.update(channel_min=round(min(per_inst), 1), channel_mean=round(mu, 1),
                               channel_max=round(max(per_inst), 1), max_over_mean=round(max(per_inst) / mu, 3),
                               cv=round(statistics.pstdev(per_inst) / mu, 4))
            per.setdefault(key, {})[cname] = row
        doc[os.path.basename(d)] = {"csv_columns": cols, "kernels": per}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1)[:6000])


if __name__ == "__main__":
    main()
