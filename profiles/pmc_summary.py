"""Summarise rocprofv3 --pmc passes (profiles/r03m_run.sh) into one JSON document: for every pass
directory given, per (kernel, grid) the mean of each counter per dispatch, plus derived figures
where the pass holds their inputs.  Usage: python profiles/pmc_summary.py OUT.json DIR [DIR ...]

Units, from `rocprofv3 -L` on the box (profiles/r03m/counters_avail.txt): SQ_WAVE_CYCLES,
SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_VALU and SQ_BUSY_CU_CYCLES are quad-cycles summed over the shader
engines; SQ_BUSY_CYCLES and SQ_CYCLES are cycles per SE summed over the 32 SEs; GRBM_GUI_ACTIVE is
summed over the 8 XCDs (it reads 8x the kernel's duration in cycles).  E = GRBM_GUI_ACTIVE / 8 is
the dispatch's elapsed cycles.  Derived:
  valu_busy      = 4 * SQ_ACTIVE_INST_VALU / (4 SIMDs x 256 CUs) / E
  waves_resident = 4 * SQ_WAVE_CYCLES / E              (mean waves alive on the chip)
  wave_cycles    = 4 * SQ_WAVE_CYCLES / SQ_WAVES         (mean wave lifetime in cycles)
  wait_frac      = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (share of wave time waiting on a counter)
  sq_busy        = SQ_BUSY_CYCLES / SQ_CYCLES
  valu_per_wave  = SQ_INSTS_VALU / SQ_WAVES, vmem_rd_per_wave = SQ_INSTS_VMEM_RD / SQ_WAVES"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

CUS, SIMDS, XCDS = 256, 4, 8


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel)<([^>]*)>", name)
    if m:
        return "%s<%s>" % (m.group(1), m.group(2))
    m = re.search(r"(\w+_kernel)I", name)  # mangled
    return m.group(1) + name[m.end() - 1:][:60] if m else name[:120]


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    doc = {}
    for d in dirs:
        acc = defaultdict(lambda: defaultdict(list))
        for r in load(d):
            key = "%s grid=%s" % (short(r.get("Kernel_Name", "")), r.get("Grid_Size", r.get("Grid_Size_X", "?")))
            # one row per (dispatch, counter); sum the dimension rows of one dispatch first
            acc[key][(r.get("Counter_Name"), r.get("Dispatch_Id"))].append(float(r.get("Counter_Value", 0) or 0))
        per = {}
        for key, cnt in acc.items():
            by_counter = defaultdict(list)
            for (cname, _), vals in cnt.items():
                by_counter[cname].append(sum(vals))
            means = {c: sum(v) / len(v) for c, v in by_counter.items()}
            n_disp = max(len(v) for v in by_counter.values())
            if n_disp < 3 or "wsum" not in key:  # the reduce kernels only (not torch's init kernels)
                continue
            g = means.get("GRBM_GUI_ACTIVE")
            g = g / XCDS if g else None
            der = {}
            if g:
                der["elapsed_cycles"] = round(g)
            if g and "SQ_ACTIVE_INST_VALU" in means:
                der["valu_busy"] = round(4 * means["SQ_ACTIVE_INST_VALU"] / (SIMDS * CUS) / g, 4)
            if g and "SQ_WAVE_CYCLES" in means:
                der["waves_resident"] = round(4 * means["SQ_WAVE_CYCLES"] / g, 1)
            if means.get("SQ_WAVE_CYCLES") and means.get("SQ_WAVES"):
                der["wave_cycles"] = round(4 * means["SQ_WAVE_CYCLES"] / means["SQ_WAVES"])
            if means.get("SQ_CYCLES") and "SQ_BUSY_CYCLES" in means:
                der["sq_busy"] = round(means["SQ_BUSY_CYCLES"] / means["SQ_CYCLES"], 4)
            if "SQ_WAIT_INST_ANY" in means and means.get("SQ_WAVE_CYCLES"):
                der["wait_frac"] = round(means["SQ_WAIT_INST_ANY"] / means["SQ_WAVE_CYCLES"], 4)
            if means.get("SQ_WAVES"):
                for c, k in (("SQ_INSTS_VALU", "valu_per_wave"), ("SQ_INSTS_VMEM_RD", "vmem_rd_per_wave"),
                             ("SQ_INSTS_SALU", "salu_per_wave"), ("SQ_INSTS_VMEM_WR", "vmem_wr_per_wave")):
                    if c in means:
                        der[k] = round(means[c] / means["SQ_WAVES"], 2)
            per[key] = {"dispatches": n_disp, "mean": {c: round(v, 1) for c, v in sorted(means.items())},
                        "derived": der}
        doc[os.path.basename(d.rstrip("/"))] = per
    with open(out, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print(json.dumps(doc, indent=1, sort_keys=True)[:6000])


if __name__ == "__main__":
    main()
