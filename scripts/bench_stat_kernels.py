#!/usr/bin/env python3
"""Timing of the K17 / K20 / K21 / K22 device paths at the reference benchmark shapes (one GPU):
DCT 10M x 100 (dct-benchmark.json; hand-written f32-MFMA kernel vs the library GEMM it replaced),
NaiveBayes fit 2M x 100, arity 20, 10 labels (naivebayes-benchmark.json), ChiSqTest on the same
table, BinaryClassificationEvaluator over 10M scores (no reference benchmark: the LR benchmark's
row count). Prints one JSON line per case; run it under `rocprofv3 --kernel-trace --stats` to see
the kernels each path launches."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, sorted(ts)[len(ts) // 2] * 1e3


def main():
    from flink_ml_amd import Table
    from flink_ml_amd.models import ChiSqTest, NaiveBayes
    from flink_ml_amd.models.evaluation import compute_metrics
    from flink_ml_amd.ops.dct import dct_matrix, dct_rows

    which = sys.argv[1:] or ["dct", "nb", "chisq", "eval"]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    if "dct" in which:
        X = torch.rand((10_000_000, 100), generator=g, device=dev, dtype=torch.float32)
        M = dct_matrix(100).to(dev, torch.float32)
        mn, md = timed(lambda: dct_rows(X))
        ln, lm = timed(lambda: X @ M.t())
        print(json.dumps({"case": "dct 10M x 100 f32", "mfma_kernel_ms": round(mn, 3), "mfma_kernel_median_ms": round(md, 3),
                          "library_gemm_ms": round(ln, 3), "hbm_gb_s": round(8e9 / (mn * 1e-3) / 1e9, 1),
                          "tflops": round(2e11 / (mn * 1e-3) / 1e12, 1)}), flush=True)
        del X
    if "nb" in which or "chisq" in which:
        X = torch.randint(0, 20, (2_000_000, 100), generator=g, device=dev).to(torch.float32)
        y = torch.randint(0, 10, (2_000_000,), generator=g, device=dev).to(torch.float64)
        t = Table({"features": X, "label": y}, num_rows=2_000_000)
        if "nb" in which:
            mn, md = timed(lambda: NaiveBayes().fit(t))
            print(json.dumps({"case": "naivebayes fit 2M x 100 (arity 20, 10 labels)", "ms": round(mn, 3),
                              "median_ms": round(md, 3)}), flush=True)
        if "chisq" in which:
            mn, md = timed(lambda: ChiSqTest().transform(t))
            print(json.dumps({"case": "chisqtest 2M x 100 (arity 20, 10 labels)", "ms": round(mn, 3),
                              "median_ms": round(md, 3)}), flush=True)
        del X, t
    if "eval" in which:
        n = 10_000_000
        s = torch.rand(n, generator=g, device=dev, dtype=torch.float64)
        p = torch.rand(n, generator=g, device=dev) < 0.3
        w = torch.ones(n, dtype=torch.float64, device=dev)
        mn, md = timed(lambda: compute_metrics(s, p, w))
        print(json.dumps({"case": "binaryclassificationevaluator 10M scores", "ms": round(mn, 3),
                          "median_ms": round(md, 3)}), flush=True)


if __name__ == "__main__":
    main()
