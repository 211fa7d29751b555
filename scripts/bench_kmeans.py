#!/usr/bin/env python3
"""KMeans throughput on MI355X against the reference's published numbers:

* KMeans-1 (reference README): 10,000 × 10 dense, k=2, maxIter 20 → reference totalTimeMs 7148,
  inputThroughput 1398.99 records/s.
* kmeans-benchmark.json: 1M × 100, k=10, maxIter 10 (no published number).
* north-star #3 per GPU shard: 12.5M × 128 (=100M/8), k=1024, bf16.
* KMeansModel.transform 10k..50k × 10 (reference 106k..394k records/s).
Prints one JSON line per config; times the whole fit (incl. init sampling) like the reference's
netRuntime (data generation excluded: it is synthetic and device-resident here).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd import Table  # noqa: E402
from flink_ml_amd.config import dtype_policy  # noqa: E402
from flink_ml_amd.models import KMeans, KMeansModel  # noqa: E402


def run_fit(n, d, k, iters, dtype, reps=3):
    dev = torch.device("cuda")
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[dtype]
    X = torch.rand((n, d), device=dev, dtype=torch.float32).to(dt)
    t = Table({"features": X})
    with dtype_policy(dtype):
        KMeans().set_k(k).set_max_iter(1).fit(t)  # warm-up (lib load, allocator)
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(reps):
            t0 = time.perf_counter()
            m = KMeans().set_k(k).set_max_iter(iters).fit(t)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
    return best, m


def run_transform(model, n, d, dtype, reps=5):
    dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp64": torch.float64}[dtype]
    t = Table({"features": torch.rand((n, d), device="cuda", dtype=torch.float32).to(dt)})
    with dtype_policy(dtype):
        model.transform(t)
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(reps):
            t0 = time.perf_counter()
            out = model.transform(t)[0]
            out.column("prediction").sum().item()
            best = min(best, time.perf_counter() - t0)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="kmeans1,ref1m,transform,north")
    a = ap.parse_args()
    cfgs = a.configs.split(",")
    if "kmeans1" in cfgs:
        for dtype in ("fp64", "fp32"):
            s, m = run_fit(10_000, 10, 2, 20, dtype)
            print(json.dumps({"bench": "KMeans-1 fit", "n": 10000, "d": 10, "k": 2, "maxIter": 20, "dtype": dtype,
                              "totalTimeMs": round(s * 1e3, 3), "inputThroughput": round(10000 / s, 1),
                              "reference_totalTimeMs": 7148.0, "reference_inputThroughput": 1398.99,
                              "speedup": round(7148.0 / (s * 1e3), 1)}), flush=True)
    if "transform" in cfgs:
        _, m = run_fit(10_000, 10, 2, 20, "fp32", reps=1)
        ref = {10000: 106383, 20000: 138889, 30000: 315789, 40000: 287770, 50000: 393701}
        for n, r in ref.items():
            s = run_transform(m, n, 10, "fp32")
            print(json.dumps({"bench": "KMeansModel-transform", "n": n, "d": 10, "k": 2,
                              "inputThroughput": round(n / s, 1), "reference_inputThroughput": r,
                              "speedup": round(n / s / r, 1)}), flush=True)
    if "ref1m" in cfgs:
        for dtype in ("fp32", "bf16"):
            s, _ = run_fit(1_000_000, 100, 10, 10, dtype)
            print(json.dumps({"bench": "kmeans-benchmark.json fit", "n": 1000000, "d": 100, "k": 10, "maxIter": 10,
                              "dtype": dtype, "totalTimeMs": round(s * 1e3, 3),
                              "inputThroughput": round(1e6 / s, 1)}), flush=True)
    if "north" in cfgs:
        n = 12_500_000
        s, _ = run_fit(n, 128, 1024, 10, "bf16", reps=1)
        flops = 2.0 * n * 1024 * 128 * 10
        print(json.dumps({"bench": "KMeans north-star shard (1 GPU of 8)", "n": n, "d": 128, "k": 1024,
                          "maxIter": 10, "dtype": "bf16", "totalTimeMs": round(s * 1e3, 2),
                          "ms_per_iter": round(s * 1e3 / 10, 3), "samples_per_s": round(n * 10 / s, 1),
                          "distance_tflops": round(flops / s / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
