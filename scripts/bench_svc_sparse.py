#!/usr/bin/env python3
"""LinearSVC on sparse (CSR) features — BASELINE.json north-star #4 (50M × 1M sparse, 8 GPUs).

One GPU runs one shard of that job: rows/8 rows of 1M-wide CSR vectors (``--nnz`` non-zeros per
row, uniform random columns), per-GPU batch 100k, hinge loss (LIB/common/lossfunc/HingeLoss.java).
A round = CSR loss+gradient kernel (wave per row: gathered dot, scatter-add of mult·x into the
dense 1M gradient), the (d+2) feedback all-reduce (one-shot xGMI on N GPUs), the update kernel —
captured in a hipGraph. Prints one JSON line: µs per round and samples/s.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer  # noqa: E402
from flink_ml_amd.parallel import comm  # noqa: E402
from flink_ml_amd.parallel.context import init_distributed  # noqa: E402
from flink_ml_amd.table import SparseColumn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50_000_000 // 8, help="rows of this GPU's shard")
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--nnz", type=int, default=64, help="non-zeros per row")
    ap.add_argument("--batch", type=int, default=100_000, help="per-GPU batch")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--sweep", default="", help="A/B grid caps, e.g. '65535:1024,4096:1024' (fwd:bwd)")
    a = ap.parse_args()
    ctx = init_distributed()
    dev = ctx.device
    g = torch.Generator(device=dev).manual_seed(7 + ctx.rank)
    n, k = a.rows, a.nnz
    indptr = torch.arange(0, (n + 1) * k, k, dtype=torch.int64, device=dev)
    idx = torch.randint(0, a.dim, (n, k), generator=g, device=dev, dtype=torch.int32)
    idx, _ = torch.sort(idx, dim=1)
    vals = torch.rand((n * k,), generator=g, device=dev, dtype=torch.float32)
    X = SparseColumn(indptr, idx.reshape(-1), vals, a.dim)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).to(torch.float32)
    world = ctx.world_size
    sgd = SGD(max_iter=10 ** 9, learning_rate=0.1, global_batch_size=a.batch * world, tol=0.0)
    tr = DeviceGlmTrainer(sgd, np.zeros(a.dim), X, y, None, "hinge", use_graph=True)
    tr.rounds_per_graph = 5
    if a.sweep:
        from flink_ml_amd.ops import glm as gk

        for cfg in a.sweep.split(","):
            f, b = (int(v) for v in cfg.split(":"))
            gk.set_csc_tuning(f, b)
            tr.graphs.clear()
            tr.run_rounds(a.warmup)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.run_rounds(a.steps)
            torch.cuda.synchronize()
            print(json.dumps({"fwd_cap": f, "bwd_cap": b, "us_per_round": round((time.perf_counter() - t0) / a.steps * 1e6, 2)}),
                  flush=True)
        gk.set_csc_tuning(0, 0)
        tr.graphs.clear()
    tr.run_rounds(a.warmup)
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    tr.run_rounds(a.steps)
    torch.cuda.synchronize()
    comm.barrier()
    el = comm.all_reduce_scalar(time.perf_counter() - t0, "max")
    assert tr.running() and tr.rounds_executed() >= a.warmup + a.steps
    if ctx.rank == 0:
        print(json.dumps({"bench": "LinearSVC sparse CSR", "n_gpus": world, "rows_per_gpu": n, "dim": a.dim,
                          "nnz_per_row": k, "per_gpu_batch": a.batch, "us_per_round": round(el / a.steps * 1e6, 2),
                          "samples_per_s": round(a.batch * world * a.steps / el)}), flush=True)


if __name__ == "__main__":
    main()
