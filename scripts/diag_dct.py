#!/usr/bin/env python3
"""A/B of the DCT kernel's pipeline at 10M x 100: full, no MFMAs, no loads, no stores, and
blocks-per-CU caps (ops/dct.set_diag). One JSON line per variant."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from flink_ml_amd.ops import dct

    X = torch.rand((10_000_000, 100), device="cuda", dtype=torch.float32)
    for diag, per_cu in [(0, 0), (1, 0), (2, 0), (4, 0), (3, 0), (5, 0), (6, 0), (0, 1), (0, 2), (1, 1), (1, 2)]:
        dct.set_diag(diag, per_cu)
        dct.dct_rows(X)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            dct.dct_rows(X)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(json.dumps({"diag": diag, "per_cu": per_cu, "ms": round(min(ts) * 1e3, 3)}), flush=True)
    dct.set_diag(0, 0)


if __name__ == "__main__":
    main()
