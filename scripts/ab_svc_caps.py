#!/usr/bin/env python3
"""A/B of the sparse SVC round's layouts — backward: untiled / row-sorted column tiles of ET
entries (glm.CSC_TILE); forward: row-group kernel / row-block × column-split cells with S splits
(glm.CELLS, glm.CELL_SPLITS) — at the svc_sparse
shard shape (scale 0.125: 6.25M x 1M, 64 nnz/row, batch 100k): steady
rounds of a warmed trainer, interleaved repeats. One JSON line per (tile, bwd_cap, repeat). (Round 5 also measured a forward taking 2/4/8 rows per
lane group: 0.0943-0.0977 ms vs 0.0899 for one row; removed.)"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import native
    from flink_ml_amd.parallel.context import init_distributed
    from flink_ml_amd.table import SparseColumn

    ctx = init_distributed()
    native.kernels()
    dev = ctx.device
    n, dim, nnz = 6_250_000, 1_000_000, 64
    g = torch.Generator(device=dev).manual_seed(7)
    idx = torch.empty((n, nnz), dtype=torch.int32, device=dev)
    for s in range(0, n, 1 << 20):
        e = min(s + (1 << 20), n)
        idx[s:e] = torch.sort(torch.randint(0, dim, (e - s, nnz), generator=g, device=dev, dtype=torch.int32), 1).values
    indptr = torch.arange(0, (n + 1) * nnz, nnz, dtype=torch.int64, device=dev)
    vals = torch.rand((n * nnz,), generator=g, device=dev, dtype=torch.float32)
    X = SparseColumn(indptr, idx.reshape(-1), vals, dim)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).to(torch.float32)
    lib = native.kernels()
    from flink_ml_amd.ops import glm as gk

    trainers = {}
    cfgs = [(32768, 8, 1, 0, 11), (32768, 8, 1, -1, 0), (32768, 8, 1, 10, 11), (32768, 8, 1, 16, 11),
            (32768, 8, 1, 6, 10)]
    if len(sys.argv) > 1 and sys.argv[1] == "--layouts":  # (round-5 layout sweep)
        cfgs = [(0, 8, 0, 0, 11), (32768, 8, 0, 0, 11), (32768, 8, 1, 0, 11), (32768, 16, 1, 0, 11)]
    if len(sys.argv) > 1 and sys.argv[1] == "--auto":  # tiles alone vs tiles + cells (automatic shape)
        cfgs = [(32768, 8, 1, 0, 11), (32768, 8, 1, -1, 0)]
    if len(sys.argv) > 2 and sys.argv[1] == "--splits":  # e.g. --splits 1 (one config: per-kernel profiles)
        cfgs = [(32768, 8, 1, int(v), 11) for v in sys.argv[2].split(",")]
    for tile, hdiv, spread, splits, rbb in cfgs:
        gk.CSC_TILE = tile
        gk.TILE_HEAVY_DIV = hdiv
        gk.TILE_SPREAD = bool(spread)
        gk.CELLS = splits != 0  # the cell forward with this many column splits (0: row-group forward)
        gk.CELL_SPLITS = max(0, splits)  # (-1: the automatic choice)
        gk.CELL_RBB = rbb or None  # (0: the automatic choice)
        tr = DeviceGlmTrainer(SGD(max_iter=10 ** 8, learning_rate=0.1, global_batch_size=100_000, tol=0.0),
                              np.zeros(dim), X, y, None, "hinge", use_graph=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.csc.ensure(range(tr.csc.P))
        torch.cuda.synchronize()
        print(json.dumps({"tile": tile, "heavy_div": hdiv, "spread": spread, "splits": splits, "S": getattr(tr.csc, "S", 0), "rbb": tr.csc.rbb, "cells": tr.csc.cells, "cmax": tr.csc.cmax, "EB": tr.csc.EB,
                          "tiles_max": int(tr.csc.ntiles.max()) if tr.csc.ET else 0,
                          "build_ms": round((time.perf_counter() - t0) * 1e3, 1), "batches": tr.csc.P}), flush=True)
        trainers[(tile, hdiv, spread, splits, rbb)] = tr
    # (the cell trainers twice: blocks in launch order / XCD-aware split-major order)
    cases = [(k, x) for k in trainers for x in ((0, 1) if trainers[k].csc.cells else (0,))]
    for rep in range(2):
        for key, xcd in cases:
            tr = trainers[key]
            lib.fmlx_glm_set_cell_xcd(xcd)
            tr.run_rounds(20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr.run_rounds(200)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 200 * 1e3
            print(json.dumps({"tile": key[0], "heavy_div": key[1], "spread": key[2], "splits": key[3], "rbb": key[4], "xcd": xcd, "rep": rep,
                              "ms_per_round": round(ms, 4)}), flush=True)
    lib.fmlx_glm_set_cell_xcd(0)



if __name__ == "__main__":
    main()
