#!/usr/bin/env python3
"""Runs only the fused KNN kernel (for rocprofv3 --kernel-trace / --pmc passes):
``--cfg nq,n,d,k`` (default 100000,100000,100,5), ``--reps`` launches after one warm-up."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.ops import knn as ko  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="100000,100000,100,5")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--segments", type=int, default=0)
    a = ap.parse_args()
    nq, n, d, k = (int(x) for x in a.cfg.split(","))
    g = torch.Generator(device="cuda").manual_seed(0)
    Q = torch.randn((nq, d), device="cuda", generator=g)
    T = torch.randn((n, d), device="cuda", generator=g)
    pack = ko.TrainPack(T, (T * T).sum(1))
    ko.fused_topk(Q, pack, k, segments=a.segments)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        ko.fused_topk(Q, pack, k, segments=a.segments)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    S = a.segments or ko.fused_segments(nq, n, k, ko._slots(k, pack.dp, Q.device))
    print("cfg=%s S=%d ms=%.3f tflops=%.1f" % (a.cfg, S, ms, 2.0 * nq * n * d / ms / 1e9), flush=True)


if __name__ == "__main__":
    main()
