#!/usr/bin/env python3
"""Out-of-core LR at the flagship shape (10M x 1000 bf16 = 20 GB, 100k batch) on one GPU with an
HBM budget below the data size (``--budget``, default 8G): the leading batches stay resident, the
rest stream from the pinned host cache through the device ring (common/outofcore.py).

Prints one JSON line: ms per round of the streamed fit, its H2D bandwidth, the resident / streamed
batch split, the same rounds on the fully resident trainer, and the coefficient difference
between the two (same kernel, same batch order: expected 0 up to float-atomic ordering).
Run under ``rocprofv3 --kernel-trace --memory-copy-trace --output-format csv`` and
``scripts/trace_overlap.py`` for the copy / kernel overlap.
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
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=100_000)
    ap.add_argument("--budget", default="8G")
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--skip-resident", action="store_true")
    a = ap.parse_args()
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.common.outofcore import StreamedGlmTrainer, parse_bytes
    from flink_ml_amd.ops import native
    from flink_ml_amd.parallel.context import init_distributed

    ctx = init_distributed()
    native.kernels()
    dev = ctx.device
    n, d = a.rows, a.dim
    g = torch.Generator(device=dev).manual_seed(3)
    Xh = torch.empty((n, d), dtype=torch.bfloat16)  # host partition (the data is generated on the GPU)
    chunk = 1 << 20
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        Xh[s:e].copy_(torch.rand((e - s, d), generator=g, device=dev).to(torch.bfloat16))
    w_true = torch.randn(d, generator=g, device=dev)
    y = torch.empty(n, dtype=torch.float32, device=dev)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        y[s:e] = ((Xh[s:e].to(dev).float() - 0.5) @ w_true > 0).float()
    torch.cuda.synchronize()
    sgd = SGD(max_iter=a.rounds, learning_rate=0.1, global_batch_size=a.batch, tol=0.0)
    budget = parse_bytes(a.budget)
    t0 = time.perf_counter()
    st = StreamedGlmTrainer(sgd, np.zeros(d), Xh, y, None, "logistic", dev, budget)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    # warm: one epoch's worth of rounds is not needed; a few rounds bring up the copy engines
    t0 = time.perf_counter()
    coef_s = st.fit()
    torch.cuda.synchronize()
    fit_s = time.perf_counter() - t0
    stats = st.store.stats()
    h2d = st.ring.h2d_bytes if st.ring is not None else 0
    out = {"metric": "out-of-core LR rounds", "rows": n, "dim": d, "dtype": "bf16", "batch": a.batch,
           "hbm_budget_bytes": budget, "data_bytes": n * d * 2, "rounds": a.rounds,
           "resident_batches": stats["resident"], "streamed_batches": stats["streamed"],
           "setup_s": round(setup_s, 2), "streamed_fit_ms_per_round": round(fit_s * 1e3 / a.rounds, 4),
           "h2d_gb": round(h2d / 1e9, 2), "h2d_gb_per_s": round(h2d / 1e9 / fit_s, 1)}
    st.close()
    if not a.skip_resident:
        Xd = Xh.to(dev)
        tr = DeviceGlmTrainer(sgd, np.zeros(d), Xd, y, None, "logistic")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        coef_r = tr.fit()
        torch.cuda.synchronize()
        out["resident_fit_ms_per_round"] = round((time.perf_counter() - t0) * 1e3 / a.rounds, 4)
        out["coef_max_abs_diff"] = float(np.abs(coef_s - coef_r).max())
        out["coef_max_abs"] = float(np.abs(coef_r).max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
