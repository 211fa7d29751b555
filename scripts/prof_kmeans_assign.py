#!/usr/bin/env python3
"""Runs only the MFMA KMeans assign (north-star shard shape by default) for rocprofv3 passes:
``--n --d --k --reps``; prints ms and TFLOP/s per call."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.ops import kmeans as kk  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=12_500_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--sched", type=int, default=1, help="assign schedule (ops/kmeans.py ASSIGN_SCHED: 1 pipelined, 0 plain)")
    a = ap.parse_args()
    from flink_ml_amd.ops import native

    kk.set_assign_sched(a.sched)
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.rand((a.n, a.d), device="cuda", generator=g).to(torch.bfloat16)
    C = torch.rand((a.k, a.d), device="cuda", generator=g)
    cb = kk.CentroidBuffers(a.k, a.d, X.device, torch.float32)
    cb.set(C)
    out = torch.empty(a.n, dtype=torch.int32, device="cuda")
    kk.set_assign_sched(0)
    ref = kk.assign(X, cb, "euclidean").clone()
    kk.set_assign_sched(a.sched)
    kk.assign(X, cb, "euclidean", out)
    same = bool(torch.equal(out, ref))
    # rows whose label differs from the plain kernel's: count, and the worst distance gap
    # relative to the full distance (fp32 torch on the same bf16 operands)
    diff = (out != ref).nonzero().flatten()
    gap = 0.0
    if diff.numel():
        Xd = X[diff[:100000]].float()
        Cf = C.to(torch.bfloat16).float()
        d = (Xd ** 2).sum(1, keepdim=True) + (Cf ** 2).sum(1)[None, :] - 2.0 * Xd @ Cf.T
        g1 = d.gather(1, out[diff[:100000]].long()[:, None]).squeeze(1)
        g0 = d.gather(1, ref[diff[:100000]].long()[:, None]).squeeze(1)
        gap = float(((g1 - g0).abs() / d.min(1).values.abs().clamp_min(1e-30)).max())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        kk.assign(X, cb, "euclidean", out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print("sched=%d n=%d d=%d k=%d ms=%.3f tflops=%.1f labels_match_plain=%s differ=%d max_rel_gap=%.2e"
          % (a.sched, a.n, a.d, a.k, ms, 2.0 * a.n * a.k * a.d / ms / 1e9, same, int(diff.numel()), gap), flush=True)


if __name__ == "__main__":
    main()
