#!/usr/bin/env python3
"""Per-phase split of the multi-rank sparse SVC round (scripts/bench_north.py --config svc_sparse
on N ranks): for K rounds of a warmed trainer, device events around the column-major round
(forward + backward → the rank's [d + 2] feedback), the feedback all-reduce (xGMI two-shot for
the 4 MB row), and the update kernel, plus host wall time per round. Launch under
torch.distributed.run (ranks may share one GPU: FMLX_BACKEND=gloo FMLX_XGMI=force). Rank 0 prints
one JSON line with every rank's medians."""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer  # noqa: E402
from flink_ml_amd.ops import glm as gk  # noqa: E402
from flink_ml_amd.parallel import comm  # noqa: E402
from flink_ml_amd.parallel.context import init_distributed  # noqa: E402
from flink_ml_amd.table import SparseColumn  # noqa: E402


def main(rows_per_rank=125_000, dim=1_000_000, nnz=64, batch=100_000, K=40):
    ctx = init_distributed()
    dev = ctx.device
    g = torch.Generator(device=dev).manual_seed(7 + ctx.rank)
    n = rows_per_rank
    idx = torch.sort(torch.randint(0, dim, (n, nnz), generator=g, device=dev, dtype=torch.int32), dim=1).values
    indptr = torch.arange(0, (n + 1) * nnz, nnz, dtype=torch.int64, device=dev)
    vals = torch.rand((n * nnz,), generator=g, device=dev, dtype=torch.float32)
    X = SparseColumn(indptr, idx.reshape(-1), vals, dim)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).to(torch.float32)
    gb = batch * ctx.world_size
    tr = DeviceGlmTrainer(SGD(max_iter=10 ** 8, learning_rate=0.1, global_batch_size=gb, tol=0.0), np.zeros(dim), X, y,
                          None, "hinge")
    assert tr.csc is not None
    tr.csc.ensure(range(tr.csc.P))
    tr.run_rounds(5)
    torch.cuda.synchronize()
    s = tr.sgd
    ph = {"round_kernels_ms": [], "allreduce_ms": [], "update_ms": [], "host_ms": []}
    for _ in range(K):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        t0 = time.perf_counter()
        ev[0].record()
        gk.csc_round(tr.csc, tr.indptr, tr.indices, tr.values, tr.y, tr.w, tr.coef, tr.n, tr.d, tr.B, tr.loss,
                     tr.state, tr.mult, tr.wl, tr.feedback, False, s.max_iter, s.tol, s.learning_rate, s.reg,
                     s.elastic_net)
        ev[1].record()
        comm.all_reduce_sum(tr.feedback)
        ev[2].record()
        gk.update(tr.feedback, tr.d, tr.coef, tr.state, s.max_iter, s.tol, s.learning_rate, s.reg, s.elastic_net)
        ev[3].record()
        torch.cuda.synchronize()
        ph["host_ms"].append((time.perf_counter() - t0) * 1e3)
        ph["round_kernels_ms"].append(ev[0].elapsed_time(ev[1]))
        ph["allreduce_ms"].append(ev[1].elapsed_time(ev[2]))
        ph["update_ms"].append(ev[2].elapsed_time(ev[3]))
    # the pipelined steady state as the bench runs it (no per-round sync)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run_rounds(K)
    torch.cuda.synchronize()
    steady = (time.perf_counter() - t0) * 1e3 / K
    mine = {k: round(statistics.median(v), 4) for k, v in ph.items()}
    mine["steady_ms_per_round"] = round(steady, 4)
    mine["rank"] = ctx.rank
    out = [None] * ctx.world_size
    torch.distributed.all_gather_object(out, mine) if ctx.is_distributed else out.__setitem__(0, mine)
    if ctx.rank == 0:
        print(json.dumps({"what": "sparse SVC round split (median of %d synced rounds) + unsynced steady state" % K,
                          "world": ctx.world_size, "rows_per_rank": n, "dim": dim, "nnz_per_row": nnz,
                          "batch_per_rank": batch, "feedback_bytes": (dim + 2) * 4,
                          "backend": os.environ.get("FMLX_BACKEND", "default"),
                          "xgmi": os.environ.get("FMLX_XGMI", "default"), "ranks": out}), flush=True)


if __name__ == "__main__":
    main()
