#!/usr/bin/env python3
"""OnlineLogisticRegression (FTRL) streaming throughput — BASELINE.json north-star #5
(unbounded stream; the reference's OnlineLogisticRegression.java:83-118 FtrlIterationBody).

Feeds a stream of global mini-batches (synthetic LabeledPoint-shaped rows, device-generated)
through ``OnlineLogisticRegression.fit`` and pulls every model version: per batch one fused
local-gradient kernel, the [grad | weightSum] all-reduce (one-shot xGMI kernel on N GPUs),
the fused FTRL update and a device-resident model version. Prints one JSON line (rank 0):
samples/s over all ranks. Multi-GPU: python -m torch.distributed.run --nproc-per-node 4 ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd import Table  # noqa: E402
from flink_ml_amd.lib.classification.logisticregression import OnlineLogisticRegression  # noqa: E402
from flink_ml_amd.linalg import Vectors  # noqa: E402
from flink_ml_amd.parallel import comm  # noqa: E402
from flink_ml_amd.parallel.context import init_distributed  # noqa: E402
from flink_ml_amd.stream import StreamTable  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=1000)
    ap.add_argument("--global-batch", type=int, default=100_000)
    ap.add_argument("--batches", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    a = ap.parse_args()
    ctx = init_distributed()
    dev = ctx.device
    world, rank = ctx.world_size, ctx.rank
    local = a.global_batch // world + (1 if a.global_batch % world > rank else 0)
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    n = local * (a.batches + a.warmup)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    X = torch.rand((n, a.dim), generator=g, device=dev, dtype=torch.float32).to(dt)
    y = (X[:, :8].float().sum(1) > 4).double()
    t = Table({"features": X, "label": y})
    init = Table.from_rows([(Vectors.dense(np.zeros(a.dim)), 0)], ["coefficient", "modelVersion"])
    est = OnlineLogisticRegression().set_global_batch_size(a.global_batch).set_initial_model_data(init)
    # the rank's stream shard arrives in local mini-batches (the per-rank split of each global batch)
    model = est.fit(StreamTable.from_table(t, local))
    stream = model._stream
    for _ in range(a.warmup):
        assert stream.pull(block=True)
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    done = 0
    while done < a.batches and stream.pull(block=True):
        done += 1
    torch.cuda.synchronize()
    comm.barrier()
    el = comm.all_reduce_scalar(time.perf_counter() - t0, "max")
    last = stream.versions[-1]
    coef = last[0].values
    if rank == 0:
        print(json.dumps({"bench": "OnlineLogisticRegression FTRL stream", "n_gpus": world, "dim": a.dim,
                          "global_batch": a.global_batch, "batches": done, "dtype": a.dtype,
                          "ms_per_batch": round(el / done * 1e3, 4), "samples_per_s": round(done * a.global_batch / el),
                          "model_version": int(last[1]), "coef_finite": bool(np.all(np.isfinite(coef)))}), flush=True)


if __name__ == "__main__":
    main()
