#!/usr/bin/env python3
"""Out-of-core sparse LinearSVC at the north-star shard shape (6.25M rows x 1M columns, 64 nnz/row,
100k batch: 3.2 GB of CSR entries) with an HBM budget below the data size (``--budget``, default
1G): the leading batches stay resident, the rest stream from the pinned host cache through the
device ring (common/outofcore.py SparseBatchStore / BatchRing), every round on the bucket round.

Prints one JSON line: ms per round of the streamed fit (``--rounds``, default one pass over the
shard), the H2D bytes and rate, the resident / streamed batch split, the same rounds on the fully
resident trainer, and the coefficient difference between the two (same kernels, same batch order:
equal up to float-atomic order).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=6_250_000)
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--nnz", type=int, default=64)
    ap.add_argument("--batch", type=int, default=100_000)
    ap.add_argument("--budget", default="1G")
    ap.add_argument("--rounds", type=int, default=63)
    a = ap.parse_args()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.common.outofcore import StreamedGlmTrainer, parse_bytes
    from flink_ml_amd.ops import native
    from flink_ml_amd.parallel.context import init_distributed
    from flink_ml_amd.table import SparseColumn

    ctx = init_distributed()
    native.kernels()
    dev = ctx.device
    n, dim, nnz = a.rows, a.dim, a.nnz
    g = torch.Generator(device=dev).manual_seed(7)
    idx = torch.empty((n, nnz), dtype=torch.int32)
    vals = torch.empty((n * nnz,), dtype=torch.float32)
    chunk = 1 << 20
    for s in range(0, n, chunk):  # generated on the GPU, kept on the host
        e = min(n, s + chunk)
        blk = torch.randint(0, dim, (e - s, nnz), generator=g, device=dev, dtype=torch.int32)
        idx[s:e].copy_(torch.sort(blk, dim=1).values)
        vals[s * nnz:e * nnz].copy_(torch.rand(((e - s) * nnz,), generator=g, device=dev))
    indptr = torch.arange(0, (n + 1) * nnz, nnz, dtype=torch.int64)
    Xh = SparseColumn(indptr, idx.reshape(-1), vals, dim)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).to(torch.float32)
    torch.cuda.synchronize()
    sgd = SGD(max_iter=a.rounds, learning_rate=0.1, global_batch_size=a.batch, tol=0.0)
    budget = parse_bytes(a.budget)
    t0 = time.perf_counter()
    st = StreamedGlmTrainer(sgd, None, Xh, y, None, "hinge", dev, budget)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    got = st.fit()
    torch.cuda.synchronize()
    fit_s = time.perf_counter() - t0
    h2d = st.ring.h2d_bytes if st.ring is not None else 0
    res = {"rows": n, "dim": dim, "nnz_per_row": nnz, "batch": a.batch, "budget_bytes": budget,
           "resident_batches": st.store.R, "batches": st.store.P, "rounds": st.rounds_executed(),
           "setup_s": round(setup_s, 3), "streamed_ms_per_round": round(fit_s * 1e3 / a.rounds, 4),
           "h2d_gb": round(h2d / 1e9, 3), "h2d_gb_per_s": round(h2d / 1e9 / fit_s, 2)}
    st.close()
    del st
    torch.cuda.empty_cache()
    Xd = Xh.to(dev)
    tr = DeviceGlmTrainer(sgd, None, Xd, y, None, "hinge")
    t0 = time.perf_counter()
    ref = tr.fit()
    torch.cuda.synchronize()
    res["resident_ms_per_round"] = round((time.perf_counter() - t0) * 1e3 / a.rounds, 4)
    res["resident_path"] = "bucket" if tr.bkt is not None else "csc"
    res["max_abs_coef_diff"] = float(np.abs(got - ref).max())
    res["max_abs_coef"] = float(np.abs(ref).max())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
