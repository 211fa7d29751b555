#!/usr/bin/env python3
"""Condenses rocprofv3 CSV output into the small files committed under ``profiles/``:

* ``stats <kernel_stats.csv> <out.csv>`` — kernel name (template args kept, parameter list
  dropped), calls, total/avg/min/max µs and share of GPU time.
* ``pmc <counter_collection.csv> <out.json> <kernel-substring> [note]`` — per-dispatch medians
  of every collected counter for the matching kernel, plus derived per-wave / MFMA figures.
"""
import csv
import json
import re
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    depth, out = 0, []
    for ch in name:  # drop the parameter list: cut at the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0 and out:
            break
        out.append(ch)
    s = "".join(out)
    return re.sub(r"\s+", " ", s)[:160]


def stats(src, dst):
    rows = list(csv.DictReader(open(src)))
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct"])
        for r in rows:
            w.writerow([short(r["Name"]), r["Calls"], "%.1f" % (float(r["TotalDurationNs"]) / 1e3),
                        "%.2f" % (float(r["AverageNs"]) / 1e3), "%.2f" % (float(r["MinNs"]) / 1e3),
                        "%.2f" % (float(r["MaxNs"]) / 1e3), "%.2f" % float(r["Percentage"])])


def pmc(src, dst, match, note=""):
    med = {}
    meta = {}
    ndisp = 0
    for one in src.split(","):  # several counter passes of the same program: medians merged
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(one)):
            if match not in r["Kernel_Name"]:
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            meta = {"kernel": short(r["Kernel_Name"]), "vgpr": r.get("VGPR_Count") or r.get("Arch_VGPR_Count"),
                    "agpr": r.get("Accum_VGPR_Count"), "sgpr": r.get("SGPR_Count"),
                    "lds_bytes": r.get("LDS_Block_Size"), "grid": r.get("Grid_Size"),
                    "workgroup": r.get("Workgroup_Size")}
        names = sorted({c for d in per.values() for c in d})
        med.update({c: statistics.median(d[c] for d in per.values() if c in d) for c in names})
        ndisp = max(ndisp, len(per))
    der = {}
    if med.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in med:
        # GRBM_GUI_ACTIVE sums the 8 XCDs; 1024 SIMDs
        der["mfma_busy_share_of_simd_cycles"] = med["SQ_VALU_MFMA_BUSY_CYCLES"] / (med["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if med.get("SQ_WAVES"):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_MFMA"):
            if c in med:
                der[c.lower().replace("sq_insts_", "") + "_insts_per_wave"] = med[c] / med["SQ_WAVES"]
    if med.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in med:
                der[c.lower() + "_share_of_wave_cycles"] = med[c] / med["SQ_WAVE_CYCLES"]
    out = {"kernel": meta, "dispatches": ndisp, "pmc_median_per_dispatch": med, "derived": der, "notes": note}
    json.dump(out, open(dst, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5] if len(sys.argv) > 5 else "")
