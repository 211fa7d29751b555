#!/usr/bin/env python3
"""Probe of the first-launch-after-idle stall seen between whole SVC fits: for each idle gap and
each "what ran last" variant, N trials of {work; sync; [read-back]; sleep(gap); t0; tiny kernel;
sync; t1} — prints the distribution of t1 − t0 (host-measured launch-to-completion latency of a
1-element fill). One JSON line per variant."""
import argparse
import json
import statistics
import time

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=40)
    ap.add_argument("--gaps-ms", default="0,1,2,5")
    ap.add_argument("--heavy-gb", type=float, default=4.0, help="HBM traffic of the work before the idle gap")
    a = ap.parse_args()
    dev = torch.device("cuda")
    big = torch.empty(1 << 20, dtype=torch.float64, device=dev)
    pinned = torch.empty(1 << 20, dtype=torch.float64).pin_memory()
    tiny = torch.empty(1, device=dev)
    x = torch.randn(4096, 4096, device=dev)
    for _ in range(3):
        (x @ x).sum().item()
    keep = {}

    def fit_like():  # the previous result freed, a fresh one read back (kept), a fresh H2D
        keep.pop("r", None)
        keep["r"] = big.cpu().numpy()
        keep["h"] = torch.from_numpy(np.zeros(1 << 20)).to(dev)

    def free_prev():  # only the previous read-back's host array freed
        keep.pop("r", None)
        keep["r"] = big.cpu().numpy()

    src = torch.empty(int(a.heavy_gb * 2**30 / 8), dtype=torch.float64, device=dev)
    dst = torch.empty_like(src)

    def heavy():  # a few ms of HBM-bound work, as a whole sparse fit's transposes + rounds
        dst.copy_(src)

    def heavy_then_d2h():
        dst.copy_(src)
        keep["r"] = big.cpu().numpy()

    variants = {
        "hbm_copy": heavy,
        "hbm_copy_then_d2h_numpy": heavy_then_d2h,
        "kernel_only": lambda: None,
        "pageable_d2h_8MB": lambda: big.cpu(),
        "pinned_d2h_8MB": lambda: pinned.copy_(big),
        "d2h_numpy_kept_prev_freed": free_prev,
        "h2d_fresh_numpy_8MB": lambda: torch.from_numpy(np.zeros(1 << 20)).to(dev),
        "fit_like": fit_like,
    }
    for gap in [float(g) for g in a.gaps_ms.split(",")]:
        for name, after in variants.items():
            lat = []
            for _ in range(a.trials):
                y = x @ x  # ~0.1 ms of work
                torch.cuda.synchronize()
                after()
                torch.cuda.synchronize()
                if gap > 0:
                    time.sleep(gap / 1e3)
                t0 = time.perf_counter()
                tiny.fill_(1.0)
                torch.cuda.synchronize()
                lat.append((time.perf_counter() - t0) * 1e3)
                del y
            lat.sort()
            print(json.dumps({"gap_ms": gap, "after": name, "median_ms": round(statistics.median(lat), 3),
                              "p90_ms": round(lat[int(0.9 * len(lat))], 3), "max_ms": round(lat[-1], 3),
                              "n_over_5ms": sum(v > 5 for v in lat), "trials": len(lat)}), flush=True)


if __name__ == "__main__":
    main()
