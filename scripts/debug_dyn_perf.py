#!/usr/bin/env python3
"""Diagnostics: per-round time of the deferred fused round with the dynamic row schedule on/off,
eager launches and hipGraph replays, small round counts with progress output."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer  # noqa: E402
from flink_ml_amd.ops import glm as gk  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.rand((rows, 1000), generator=g, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 2, (rows,), generator=g, device=dev).float()
    for dyn in (0, 1):
        for graph in (False, True):
            gk.set_dyn(bool(dyn), 8)
            tr = DeviceGlmTrainer(SGD(max_iter=10 ** 6, learning_rate=0.1, global_batch_size=100_000, tol=0.0),
                                  np.zeros(1000), X, y, None, "logistic", use_graph=graph)
            tr.rounds_per_graph = 10
            for k in (1, 10, 50):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                tr.run_rounds(k)
                torch.cuda.synchronize()
                print("dyn=%d graph=%d rounds=%d us_per_round=%.1f executed=%d" % (
                    dyn, graph, k, (time.perf_counter() - t0) / k * 1e6, tr.rounds_executed()), flush=True)


if __name__ == "__main__":
    main()
