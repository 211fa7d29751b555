#!/usr/bin/env python3
"""Per-block timeline of the fused LR round at the bench shape (10M × 1000 bf16, 100k batch,
256 blocks): start, rows-done and atomics-drained stamps (s_memrealtime, 100 MHz) of every block,
summarised per round as spreads relative to the earliest block start, plus per-XCD means.

Shows how much of a round is launch skew, load imbalance (the slowest block's rows) and tail.
Usage: python scripts/trace_glm_blocks.py [--rounds 20] [--defer 1]
"""
import argparse
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer  # noqa: E402
from flink_ml_amd.ops import glm as gk  # noqa: E402

TICK_US = 0.01  # s_memrealtime runs at 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--defer", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda")
    gk.DEFER = bool(a.defer)
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.empty((a.rows, a.dim), dtype=torch.bfloat16, device=dev)
    for s in range(0, a.rows, 1 << 20):
        e = min(s + (1 << 20), a.rows)
        X[s:e] = torch.rand((e - s, a.dim), generator=g, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 2, (a.rows,), generator=g, device=dev).float()
    sgd = SGD(max_iter=10 ** 8, learning_rate=0.1, global_batch_size=a.batch, tol=0.0)
    tr = DeviceGlmTrainer(sgd, np.zeros(a.dim), X, y, None, "logistic", use_graph=False)
    tr.run_rounds(30)
    torch.cuda.synchronize()
    nb = tr.nparts
    buf = torch.zeros((nb, 4), dtype=torch.int64, device=dev)
    gk.set_trace(buf)
    rows = []
    try:
        for _ in range(a.rounds):
            buf.zero_()
            tr._launch_round(1)
            torch.cuda.synchronize()
            rows.append(buf.cpu().numpy().copy())
    finally:
        gk.set_trace(None)
    summary = []
    for t in rows:
        t0 = t[:, 0].min()
        start = (t[:, 0] - t0) * TICK_US
        done = (t[:, 1] - t0) * TICK_US
        drained = (t[:, 2] - t0) * TICK_US
        xcc = (t[:, 3] >> 32) & 0xF
        per_x = {int(x): round(float(done[xcc == x].mean()), 2) for x in sorted(set(xcc.tolist()))}
        summary.append({
            "start_max_us": round(float(start.max()), 2),
            "rows_done_min_us": round(float(done.min()), 2),
            "rows_done_med_us": round(float(np.median(done)), 2),
            "rows_done_max_us": round(float(done.max()), 2),
            "drained_max_us": round(float(drained.max()), 2),
            "block_rows_us_med": round(float(np.median(done - start)), 2),
            "rows_done_mean_by_xcd": per_x,
        })
    for s in summary:
        print(json.dumps(s))
    # is the imbalance systematic? correlation of each block's rows-done time between rounds,
    # and how often the same XCD is the slowest
    done = np.stack([(t[:, 1] - t[:, 0].min()).astype(np.float64) for t in rows])
    cc = [float(np.corrcoef(done[i], done[i + 1])[0, 1]) for i in range(len(done) - 1)]
    xcc = (rows[0][:, 3] >> 32) & 0xF
    slow = [int(max(set(xcc.tolist()), key=lambda x: done[i][xcc == x].mean())) for i in range(len(done))]
    print(json.dumps({"block_done_corr_between_rounds_median": round(statistics.median(cc), 3),
                      "slowest_xcd_per_round": slow,
                      "block_done_spread_us_if_per_block_mean_removed": round(float(
                          np.median(np.ptp(done - done.mean(0, keepdims=True), axis=1)) * TICK_US), 2)}))
    keys = ["start_max_us", "rows_done_min_us", "rows_done_med_us", "rows_done_max_us", "block_rows_us_med"]
    xm = {x: round(statistics.median(s["rows_done_mean_by_xcd"][x] for s in summary), 2)
          for x in summary[0]["rows_done_mean_by_xcd"]}
    print(json.dumps({"median_over_rounds": {k: round(statistics.median(s[k] for s in summary), 2) for k in keys},
                      "rows_done_mean_by_xcd_median": xm, "blocks": nb}))


if __name__ == "__main__":
    main()
