#!/usr/bin/env python3
"""The sparse trainer's column-major copies alone (ops/glm.py BatchCsc) at the SVC run shape:
``--batches`` batches of ``--batch`` rows × ``--nnz`` non-zeros over ``--dim`` columns, one run
(one sort) per iteration on a fresh BatchCsc — ms per run of batches, for A/Bs and rocprofv3
passes. ``--lsd`` forces the two-LSD-pass path (glm.CSC_BUCKET = False)."""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.ops import glm as gk  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=10)
    ap.add_argument("--batch", type=int, default=100_000)
    ap.add_argument("--nnz", type=int, default=64)
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lsd", action="store_true")
    a = ap.parse_args()
    gk.CSC_BUCKET = not a.lsd
    dev = torch.device("cuda")
    n = a.batches * a.batch
    g = torch.Generator(device=dev).manual_seed(1)
    idx = torch.sort(torch.randint(0, a.dim, (n, a.nnz), generator=g, device=dev, dtype=torch.int32), dim=1).values
    indptr = torch.arange(0, (n + 1) * a.nnz, a.nnz, dtype=torch.int64, device=dev)
    vals = torch.rand(n * a.nnz, generator=g, device=dev)
    idx = idx.reshape(-1)
    times = []
    for i in range(a.iters + 2):
        c = gk.BatchCsc.alloc(indptr, idx, vals, n, a.dim, a.batch)
        c._storage(c.P)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c.ensure(range(c.P))
        torch.cuda.synchronize()
        if i >= 2:
            times.append((time.perf_counter() - t0) * 1e3)
        del c
    print("csc transpose %s: %d x %d rows x %d nnz, d=%d: median %.3f ms, min %.3f ms" % (
        "lsd" if a.lsd else "bucket", a.batches, a.batch, a.nnz, a.dim, statistics.median(times), min(times)))


if __name__ == "__main__":
    main()
