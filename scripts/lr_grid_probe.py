#!/usr/bin/env python3
"""One rank of the LR flagship round (10M x 1000 bf16, batch 100k) with the round grid capped
at 64 / 128 / default blocks: how much of a shared-GPU rehearsal's round (two ranks of 128 blocks,
profiles/r5/rehearsal_2rank_1gpu_overlap.json) is the halved grid alone. One JSON line per cap:
µs per round over 200 graph-replayed rounds."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk
    from flink_ml_amd.ops import native
    from flink_ml_amd.parallel.context import init_distributed

    ctx = init_distributed()
    native.kernels()
    dev = ctx.device
    n, d = 10_000_000, 1000
    X = torch.empty((n, d), dtype=torch.bfloat16, device=dev)
    g = torch.Generator(device=dev).manual_seed(5)
    for s in range(0, n, 1 << 20):
        e = min(n, s + (1 << 20))
        X[s:e] = torch.rand((e - s, d), generator=g, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).float()
    base = gk.max_round_blocks
    for cap in (0, 128, 64):
        gk.max_round_blocks = (lambda c=cap: c) if cap else base
        tr = DeviceGlmTrainer(SGD(max_iter=10 ** 6, learning_rate=0.1, global_batch_size=100_000, tol=0.0),
                              np.zeros(d), X, y, None, "logistic")
        tr.run_rounds(50)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.run_rounds(200)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / 200 * 1e6
        print(json.dumps({"grid_cap": cap or "default", "blocks": tr.nparts, "us_per_round": round(us, 2)}), flush=True)
    gk.max_round_blocks = base


if __name__ == "__main__":
    main()
