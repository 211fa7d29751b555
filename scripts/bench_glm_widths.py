#!/usr/bin/env python3
"""Dense SGD rounds across row widths (ms per round, effective HBM rate of the batch read):
which kernel each width takes (one-wave fused round / wide-row fused round / GEMV fallback) and
how fast. ``FMLX_GLM_WIDE_FUSED=0`` sends the wide widths to the GEMV path for an A/B.
One JSON line per (dtype, d)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("bf16", 1000), ("bf16", 2048), ("bf16", 4096), ("bf16", 8192), ("bf16", 16384), ("fp32", 1001),
          ("fp32", 4096), ("fp32", 16384), ("fp64", 1000), ("fp64", 3000)]
DT = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}


def main():
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import native

    native.kernels()
    dev = torch.device("cuda")
    B = 100_000
    rounds = int(os.environ.get("ROUNDS", "40"))
    for name, d in SHAPES:
        dt = DT[name]
        n = 4 * B
        g = torch.Generator(device=dev).manual_seed(d)
        X = torch.empty((n, d), dtype=dt, device=dev)
        for s in range(0, n, 50_000):
            X[s:s + 50_000] = torch.rand((min(50_000, n - s), d), generator=g, device=dev).to(dt)
        y = (torch.rand(n, generator=g, device=dev) > 0.5).to(torch.float64 if dt == torch.float64 else torch.float32)
        sgd = SGD(max_iter=10 ** 8, learning_rate=0.1, global_batch_size=B, tol=0.0)
        tr = DeviceGlmTrainer(sgd, np.zeros(d), X, y, None, "logistic", use_graph=False)
        kind = "fused" if tr.layout is not None else ("wide_fused" if tr.wide_fused else "gemv")
        tr.run_rounds(5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.run_rounds(rounds)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / rounds * 1e3
        gbs = B * tr.X.shape[1] * tr.X.element_size() / ms / 1e6
        print(json.dumps({"dtype": name, "d": d, "kernel": kind, "padded_d": int(tr.X.shape[1]),
                          "blocks": int(tr.nparts), "ms_per_round": round(ms, 4), "batch_GB_per_s": round(gbs, 1)}),
              flush=True)
        del tr, X, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
