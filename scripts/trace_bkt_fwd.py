#!/usr/bin/env python3
"""Per-block phase timeline of the bucket round's forward (glm_sparse.hip glm_bkt_fwd_scatter_kernel)
at the SVC shape (1M columns, 64 nnz/row, 100k-row batches): s_memrealtime stamps (100 MHz) at
block entry (0), wave 0's entries + bookkeeping rows landed (6), coefficient gathers landed and the
products staged (1), row ids filled (2), row dots + loss done (3), records staged in LDS (4),
record stores issued (5), summarised per round relative to the earliest block entry.

Usage: python scripts/trace_bkt_fwd.py [--rounds 5] [--rows 1000000]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TICK_US = 0.01
PHASES = [("entries_bookkeeping", 0, 6), ("gathers", 6, 1), ("row_ids", 1, 2), ("dots_loss", 2, 3),
          ("staging", 3, 4), ("store_issue", 4, 5)]


def q(x, p):
    return round(float(np.percentile(x, p)), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--rows", type=int, default=1_000_000)
    a = ap.parse_args()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk
    from flink_ml_amd.table import SparseColumn

    dev = torch.device("cuda")
    n, dim, nnz = a.rows, 1_000_000, 64
    g = torch.Generator(device=dev).manual_seed(7)
    idx = torch.sort(torch.randint(0, dim, (n, nnz), generator=g, device=dev, dtype=torch.int32), 1).values
    indptr = torch.arange(0, (n + 1) * nnz, nnz, dtype=torch.int64, device=dev)
    vals = torch.rand((n * nnz,), generator=g, device=dev, dtype=torch.float32)
    X = SparseColumn(indptr, idx.reshape(-1), vals, dim)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).to(torch.float32)
    gk.TILE_MIN_VISITS = 10 ** 9
    tr = DeviceGlmTrainer(SGD(max_iter=10 ** 8, learning_rate=0.1, global_batch_size=100_000, tol=0.0),
                          None, X, y, None, "hinge", use_graph=False)
    assert tr.bkt is not None
    tr.run_rounds(20)
    torch.cuda.synchronize()
    blocks = -(-100_000 // tr.bkt.rb)
    buf = torch.zeros((blocks, 8), dtype=torch.int64, device=dev)
    rows = []
    gk.set_bkt_trace(buf)
    try:
        for _ in range(a.rounds):
            buf.zero_()
            tr.run_rounds(1)
            torch.cuda.synchronize()
            rows.append(buf.cpu().numpy().copy())
    finally:
        gk.set_bkt_trace(None)
    for t in rows:
        live = t[:, 0] > 0
        t = t[live]
        t0 = t[:, 0].min()
        st = [(t[:, i] - t0) * TICK_US for i in range(7)]
        ent, end = st[0], st[5]
        # blocks resident at once: entries before the first block's end
        first_end = float(end.min())
        print(json.dumps({
            "blocks": int(live.sum()), "rb": tr.bkt.rb,
            "entry_p50_p90_max_us": [q(ent, 50), q(ent, 90), round(float(ent.max()), 2)],
            "resident_at_first_end": int((ent < first_end).sum()),
            "span_us": round(float(end.max()), 2),
            "block_us_p50_p90": [q(end - ent, 50), q(end - ent, 90)],
            "phase_p50_us": {k: q(st[b] - st[a], 50) for k, a, b in PHASES},
            "phase_p90_us": {k: q(st[b] - st[a], 90) for k, a, b in PHASES},
        }), flush=True)


if __name__ == "__main__":
    main()
