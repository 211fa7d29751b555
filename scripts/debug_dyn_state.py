#!/usr/bin/env python3
"""Diagnostics of the dynamic row schedule's termination: per (block, wave) exit chunk number,
walk steps over empty chunks, spin-cap exits and the block's exh / inflight / lastv, one round."""
import collections
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer  # noqa: E402
from flink_ml_amd.ops import glm as gk, native  # noqa: E402


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.rand((400_000, 1000), generator=g, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 2, (400_000,), generator=g, device=dev).float()
    gk.set_dyn(True, 8)
    tr = DeviceGlmTrainer(SGD(max_iter=100, learning_rate=0.1, global_batch_size=100_000, tol=0.0), np.zeros(1000), X,
                          y, None, "logistic", use_graph=False)
    lib = native.kernels()
    for r in range(3):
        buf = torch.full((tr.nparts * 8 * 8,), -7, dtype=torch.int32, device=dev)
        lib.fmlx_glm_set_dyn_debug2(native.ptr(buf))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr._launch_round(1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        lib.fmlx_glm_set_dyn_debug2(None)
        b = buf.view(tr.nparts, 8, 8).cpu().numpy()
        print(json.dumps({"round": r, "ms": round(dt * 1e3, 2),
                          "exit_q": collections.Counter(b[:, :, 0].ravel().tolist()).most_common(6),
                          "walk_steps_max": int(b[:, :, 1].max()), "walk_steps_mean": float(b[:, :, 1].mean()),
                          "caps_total": int(b[:, :, 2].sum()), "exh": collections.Counter(b[:, 0, 3].tolist()).most_common(3),
                          "inflight": collections.Counter(b[:, :, 4].ravel().tolist()).most_common(4),
                          "lastv": collections.Counter(b[:, 0, 5].tolist()).most_common(6),
                          "block0": b[0].tolist()}), flush=True)


if __name__ == "__main__":
    main()
