#!/usr/bin/env python3
"""Steady sparse-SVC rounds at the svc_sparse shard shape (6.25M x 1M, 64 nnz/row, batch 100k)
for kernel traces / counters: one warmed trainer (every batch transposed; glm.CSC_TILE picks the
backward layout), then ``--rounds`` rounds.

  rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python3 scripts/prof_svc_round.py
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
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--rows", type=int, default=6_250_000)
    args = ap.parse_args()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import native
    from flink_ml_amd.parallel.context import init_distributed
    from flink_ml_amd.table import SparseColumn

    ctx = init_distributed()
    native.kernels()
    dev = ctx.device
    n, dim, nnz = args.rows, 1_000_000, 64
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
    t0 = time.perf_counter()
    tr.run_rounds(args.rounds)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.rounds * 1e3
    print(json.dumps({"tile": tr.csc.ET, "rounds": args.rounds, "ms_per_round": round(ms, 4)}), flush=True)


if __name__ == "__main__":
    main()
