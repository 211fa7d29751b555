#!/usr/bin/env python3
"""Diagnostics: where the sparse trainer's constructor spends its host time (statement timers
around a replica of DeviceGlmTrainer.__init__'s steps on the SVC north-star shard)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer  # noqa: E402
from flink_ml_amd.table import SparseColumn  # noqa: E402


def main():
    dev = torch.device("cuda")
    n, dim, nnz = 6_250_000, 1_000_000, 64
    g = torch.Generator(device=dev).manual_seed(7)
    idx = torch.randint(0, dim, (n, nnz), generator=g, device=dev, dtype=torch.int32)
    indptr = torch.arange(0, (n + 1) * nnz, nnz, dtype=torch.int64, device=dev)
    vals = torch.rand((n * nnz,), generator=g, device=dev)
    X = SparseColumn(indptr, idx.reshape(-1), vals, dim)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).float()
    torch.cuda.synchronize()
    for rep in range(3):
        sgd = SGD(max_iter=10, learning_rate=0.1, global_batch_size=100_000, tol=0.0)
        marks = []
        orig = time.perf_counter

        def mark(tag):
            torch.cuda.synchronize()
            marks.append((tag, orig()))

        mark("start")
        tr = DeviceGlmTrainer(sgd, np.zeros(dim), X, y, None, "hinge")
        marks.append(("ctor(host)", orig()))
        mark("ctor(sync)")
        tr.csc.ensure_rounds(0, 10)
        mark("transpose")
        tr.fit()
        mark("fit")
        print(rep, " ".join("%s=%.2fms" % (marks[i][0], (marks[i][1] - marks[i - 1][1]) * 1e3)
                            for i in range(1, len(marks))), flush=True)
    # bench_north's sequence: a 2-round warm fit, then the timed whole fit, with per-line times of
    # the constructor (sys.settrace line events; C-level slot operations included)
    warm = DeviceGlmTrainer(SGD(max_iter=2, learning_rate=0.1, global_batch_size=100_000, tol=0.0), np.zeros(dim), X,
                            y, None, "hinge")
    warm.fit()
    del warm, tr
    torch.cuda.synchronize()
    code = DeviceGlmTrainer.__init__.__code__
    times = {}
    last = [None, 0.0]

    def tracer(frame, event, arg):
        if frame.f_code is not code:
            return None

        def local(frame, event, arg):
            now = time.perf_counter()
            if last[0] is not None:
                times[last[0]] = times.get(last[0], 0.0) + now - last[1]
            last[0] = frame.f_lineno if event == "line" else None
            last[1] = time.perf_counter()
            return local
        return local

    sys.settrace(tracer)
    t0 = time.perf_counter()
    tr = DeviceGlmTrainer(SGD(max_iter=10, learning_rate=0.1, global_batch_size=100_000, tol=0.0), np.zeros(dim), X,
                          y, None, "hinge")
    t1 = time.perf_counter()
    sys.settrace(None)
    print("ctor %.2f ms; slowest lines:" % ((t1 - t0) * 1e3))
    for ln, t in sorted(times.items(), key=lambda kv: -kv[1])[:10]:
        print("  line %d: %.3f ms" % (ln, t * 1e3))
    t0 = time.perf_counter()
    tr.fit()
    torch.cuda.synchronize()
    print("fit %.2f ms" % ((time.perf_counter() - t0) * 1e3))

if __name__ == "__main__":
    main()
