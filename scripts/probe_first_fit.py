#!/usr/bin/env python3
"""Host-side profile of the FIRST sparse-SVC whole fit of a fresh process (cumulative cProfile and
the callers of the hot built-ins), at the svc_sparse shape scaled down."""
import cProfile
import io
import os
import pstats
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
    n, dim, nnz = 800_000, 1_000_000, 64
    g = torch.Generator(device=dev).manual_seed(7)
    idx = torch.sort(torch.randint(0, dim, (n, nnz), generator=g, device=dev, dtype=torch.int32), dim=1).values
    indptr = torch.arange(0, (n + 1) * nnz, nnz, dtype=torch.int64, device=dev)
    vals = torch.rand((n * nnz,), generator=g, device=dev, dtype=torch.float32)
    X = SparseColumn(indptr, idx.reshape(-1), vals, dim)
    y = torch.randint(0, 2, (n,), generator=g, device=dev).to(torch.float32)
    torch.cuda.synchronize()
    for i in range(3):
        prof = cProfile.Profile()
        t0 = time.perf_counter()
        prof.enable()
        tr = DeviceGlmTrainer(SGD(max_iter=10, learning_rate=0.1, global_batch_size=100_000, tol=0.0), np.zeros(dim),
                              X, y, None, "hinge")
        tr.fit()
        prof.disable()
        torch.cuda.synchronize()
        print("fit %d: %.3f ms" % (i, (time.perf_counter() - t0) * 1e3), flush=True)
        if i == 0:
            s = io.StringIO()
            st = pstats.Stats(prof, stream=s).sort_stats("cumulative")
            st.print_stats(40)
            st.print_callers("copy_|compile|_process_class|exec")
            print(s.getvalue())


if __name__ == "__main__":
    main()
