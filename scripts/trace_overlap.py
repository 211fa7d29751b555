#!/usr/bin/env python3
"""Overlap of host→device copies with kernels in a rocprofv3 trace (``--kernel-trace
--memory-copy-trace --output-format csv``): how much of the H2D copy time runs while a kernel of
the same process is executing, and how much of the kernel time runs under a copy.

Usage: python scripts/trace_overlap.py <rocprof output dir> [--kernel-filter SUBSTR] [--fit-window]
(--fit-window: only copies that start between the first and last filtered kernel)
Prints one JSON line.
"""
import csv
import glob
import json
import os
import sys


def _rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def _merge(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _overlap(a, b):
    """Total length of the intersection of two merged interval lists."""
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s = max(a[i][0], b[j][0])
        e = min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    d = sys.argv[1]
    filt = None
    if "--kernel-filter" in sys.argv:
        filt = sys.argv[sys.argv.index("--kernel-filter") + 1]
    kr = _rows(os.path.join(d, "**", "*kernel_trace.csv"))
    mr = _rows(os.path.join(d, "**", "*memory_copy_trace.csv"))
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kr
            if filt is None or filt in r.get("Kernel_Name", "")]
    h2d = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in mr
           if "HOST_TO_DEVICE" in r.get("Direction", "").upper() or "H2D" in r.get("Direction", "").upper()]
    big = [c for c in h2d if c[1] - c[0] > 100_000]  # batch-sized copies (> 0.1 ms)
    if "--fit-window" in sys.argv and kern:
        # only the copies issued while the filtered kernels run (not the set-up's resident fill)
        t0, t1 = min(k[0] for k in kern), max(k[1] for k in kern)
        big = [c for c in big if c[0] >= t0 and c[0] <= t1]
    K, C = _merge(kern), _merge(big)
    ctot = sum(e - s for s, e in C)
    ktot = sum(e - s for s, e in K)
    ov = _overlap(K, C)
    span = (max(x[1] for x in K + C) - min(x[0] for x in K + C)) if K and C else 0
    print(json.dumps({
        "kernels": len(kern), "h2d_copies": len(h2d), "batch_copies": len(big),
        "h2d_ms": round(ctot / 1e6, 3), "kernel_ms": round(ktot / 1e6, 3), "span_ms": round(span / 1e6, 3),
        "kernel_time_under_copy_frac": round(ov / ktot, 4) if ktot else None,
        "copy_busy_frac_of_span": round(ctot / span, 4) if span else None,
        "mean_copy_ms": round(ctot / len(big) / 1e6, 4) if big else None,
    }))


if __name__ == "__main__":
    main()
