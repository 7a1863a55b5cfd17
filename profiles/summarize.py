"""Summarise rocprofv3 output of profiles/collect.sh into committed files:
<out>/summary/<round>_kernel_stats.csv (copy of the stats), <round>_summary.json and
pmc_traffic.json (read by bench.py for roofline.traffic once copied into profiles/)."""
import csv
import glob
import json
import os
import shutil
import sys

out_dir, rnd = sys.argv[1], sys.argv[2]
args = sys.argv[3:]
HERE = os.path.join(out_dir, "summary")  # copied into profiles/ by hand after gpurun merges it back
os.makedirs(HERE, exist_ok=True)
KERNEL = "wsum_stream_kernel"


def find(pattern):
    hits = sorted(glob.glob(os.path.join(out_dir, "**", pattern), recursive=True))
    return hits[0] if hits else None


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


summary = {"round": rnd, "bench_args": args}
stats = find("*kernel_stats.csv")
kname = None
if stats:
    shutil.copy(stats, os.path.join(HERE, "%s_kernel_stats.csv" % rnd))
    # the dominant instantiation of the reduce kernel = the north-star launches
    cands = [r for r in rows(stats) if KERNEL in r.get("Name", "")]
    if cands:
        r = max(cands, key=lambda r: float(r["TotalDurationNs"]))
        kname = r["Name"]
        summary["kernel"] = kname
        summary["calls"] = int(r["Calls"])
        summary["avg_ns"] = float(r["AverageNs"])
        summary["min_ns"] = float(r["MinNs"])
        summary["max_ns"] = float(r["MaxNs"])


def pmc(sub, counter):
    path = find(os.path.join(sub, "**", "*counter_collection.csv")) or find("*%s*counter_collection.csv" % sub)
    if path is None:
        cands = [p for p in glob.glob(os.path.join(out_dir, sub, "**", "*counter_collection.csv"), recursive=True)]
        path = cands[0] if cands else None
    if path is None:
        return None
    vals = [float(r["Counter_Value"]) for r in rows(path)
            if (r.get("Kernel_Name", "") == kname if kname else KERNEL in r.get("Kernel_Name", ""))
            and r.get("Counter_Name") == counter]
    if not vals:
        return None
    vals.sort()
    return vals[len(vals) // 2]  # median over dispatches (KB per dispatch)


fetch_kb = pmc("fetch", "FETCH_SIZE")
write_kb = pmc("write", "WRITE_SIZE")
summary["FETCH_SIZE_kb_median"] = fetch_kb
summary["WRITE_SIZE_kb_median"] = write_kb
n_peers = int(args[args.index("--peers") + 1]) if "--peers" in args else 8
params = int(args[args.index("--params") + 1]) if "--params" in args else 25_000_000
algo = (n_peers + 1) * params * 4
summary["algorithmic_bytes_per_launch"] = algo
if fetch_kb is not None and write_kb is not None:
    # gfx950: FETCH_SIZE counts half of a wide coalesced stream's bytes -> x2 (MI355X guide, HBM section)
    hbm = 2 * fetch_kb * 1024 + write_kb * 1024
    summary["hbm_bytes_per_launch"] = hbm
    summary["hbm_over_algorithmic"] = hbm / algo
    json.dump({"workload": "ns", "peers": n_peers, "params": params, "hbm_bytes_per_launch": int(hbm),
               "fetch_kb_raw": fetch_kb, "write_kb": write_kb, "correction": "FETCH_SIZE x2 (gfx950 16-B streams)",
               "source": "profiles/%s_summary.json" % rnd}, open(os.path.join(HERE, "pmc_traffic.json"), "w"), indent=1)
if "avg_ns" in summary:
    summary["achieved_GBps_from_trace"] = algo / summary["avg_ns"]
json.dump(summary, open(os.path.join(HERE, "%s_summary.json" % rnd), "w"), indent=1)
print(json.dumps(summary, indent=1))
