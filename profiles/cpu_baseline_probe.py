"""The cpu_baseline leg of bench.py alone, in a fresh process (variance across processes / boxes),
plus the host facts that move it: THP mode, NUMA nodes, the GPU's NUMA node, CPU affinity."""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def read(path):
    try:
        return open(path).read().strip()
    except OSError:
        return None


facts = {"thp": read("/sys/kernel/mm/transparent_hugepage/enabled"),
         "thp_defrag": read("/sys/kernel/mm/transparent_hugepage/defrag"),
         "numa_nodes": sorted(os.path.basename(p) for p in glob.glob("/sys/devices/system/node/node*")),
         "gpu_numa_node": [read(p) for p in glob.glob("/sys/class/drm/card*/device/numa_node")],
         "affinity_cpus": len(os.sched_getaffinity(0)),
         "cpus_by_node": {os.path.basename(p): read(p + "/cpulist") for p in glob.glob("/sys/devices/system/node/node*")}}
print(json.dumps(facts), flush=True)
cb = bench.cpu_baseline(8, 25_000_000, float(sys.argv[1]) if len(sys.argv) > 1 else 5.0)
print(json.dumps({k: cb[k] for k in ("value", "cores", "sample", "by_threads")}), flush=True)
