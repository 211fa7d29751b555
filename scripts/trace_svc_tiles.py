#!/usr/bin/env python3
"""Per-block timeline of the tiled sparse backward (glm.hip glm_csc_tile_bwd_kernel) at the SVC
shard shape (6.25M x 1M, 64 nnz/row, batch 100k): s_memrealtime stamps (100 MHz) at block entry,
after the thread's own gathers, after the block barrier (all gathers of the tile done) and after
the column pass, summarised per round relative to the earliest block entry.

Usage: python scripts/trace_svc_tiles.py [--rounds 10] [--rows 6250000]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TICK_US = 0.01


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--rows", type=int, default=6_250_000)
    a = ap.parse_args()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk
    from flink_ml_amd.table import SparseColumn

    dev = torch.device("cuda")
    n, dim, nnz = a.rows, 1_000_000, 64
    g = torch.Generator(device=dev).manual_seed(7)
    idx = torch.empty((n, nnz), dtype=torch.int32, device=dev)
    for s in range(0, n, 1 << 20):
        e = min(s + (1 << 20), n)
        idx[s:e] = torch.sort(torch.randint(0, dim, (e - s, nnz), generator=g, device=dev, dtype=torch.int32), 1).values
    indptr = torch.arange(0, (n + 1) * nnz, nnz, dtype=torch.int64, device=dev)
    vals = torch.rand((n * nnz,), generator=g, device=dev, dtype=torch.float32)
    X = SparseColumn(indptr, idx.reshape(-1), vals, dim)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).to(torch.float32)
    tr = DeviceGlmTrainer(SGD(max_iter=10 ** 8, learning_rate=0.1, global_batch_size=100_000, tol=0.0),
                          np.zeros(dim), X, y, None, "hinge", use_graph=False)
    tr.csc.ensure(range(tr.csc.P))
    tr.run_rounds(20)
    torch.cuda.synchronize()
    buf = torch.zeros((4096, 4), dtype=torch.int64, device=dev)
    nt = tr.csc.ntiles.cpu().numpy()
    rows = []
    gk.set_trace(buf)
    try:
        for _ in range(a.rounds):
            buf.zero_()
            tr.run_rounds(1)
            torch.cuda.synchronize()
            rows.append(buf.cpu().numpy().copy())
    finally:
        gk.set_trace(None)
    for t in rows:
        live = t[:, 0] > 0
        t = t[live]
        t0 = t[:, 0].min()
        ent, gat, bar, end = [(t[:, i] - t0) * TICK_US for i in range(4)]
        print(json.dumps({
            "blocks": int(live.sum()), "tiles_per_batch_median": float(np.median(nt)),
            "entry_max_us": round(float(ent.max()), 2),
            "own_gathers_done_med_us": round(float(np.median(gat)), 2),
            "barrier_med_us": round(float(np.median(bar)), 2), "barrier_max_us": round(float(bar.max()), 2),
            "end_med_us": round(float(np.median(end)), 2), "end_max_us": round(float(end.max()), 2),
            "gather_phase_med_us": round(float(np.median(bar - ent)), 2),
            "column_phase_med_us": round(float(np.median(end - bar)), 2),
        }), flush=True)


if __name__ == "__main__":
    main()
