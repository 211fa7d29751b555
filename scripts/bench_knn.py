#!/usr/bin/env python3
"""KnnModel.transform throughput on one MI355X (K3/K13; reference ``KnnModel.java:154-194``).

Compares, on the same device-resident data: the production predict (ONE fused kernel: fp32
matrix-core distances + top-k in registers, training pack cached as the model caches it), the
split path (hipBLASLt fp32 GEMM block + one ``knn.hip`` top-k scan of it) and the unfused PyTorch
chain (addmm with the norm broadcast → abs → sqrt → topk).
Prints one JSON line per config. Synthetic Gaussian data; no reference number is published.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.models.knn import knn_predict, knn_vote  # noqa: E402
from flink_ml_amd.ops import knn as ko  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    dev = torch.device("cuda")
    ap.add_argument("--configs", default="all")
    ap.add_argument("--only-fused", action="store_true", help="time only the production path (for kernel traces)")
    args = ap.parse_args()
    configs = [(100_000, 100_000, 100, 5), (100_000, 1_000_000, 64, 10), (10_000, 100_000, 100, 32),
               (10_000, 100_000, 100, 64)]
    if args.configs != "all":
        configs = [configs[int(i)] for i in args.configs.split(",")]
    for nq, n, d, k in configs:
        g = torch.Generator(device=dev).manual_seed(0)
        Q = torch.randn((nq, d), device=dev, generator=g)
        T = torch.randn((n, d), device=dev, generator=g)
        labels = torch.randint(0, 10, (n,), device=dev, generator=g).double()
        classes = torch.unique(labels)
        tn = (T * T).sum(1)

        pack = ko.TrainPack(T, tn)

        def fused():  # the production KnnModel path (pack cached per model)
            knn_predict(Q, T, tn, labels, k, pack=pack, classes=classes)

        def split():  # library GEMM block + top-k scan (the D > 128 path)
            qb = ko.query_block(n)
            for s in range(0, nq, qb):
                q = Q[s:s + qb]
                idx = ko.topk_from_products(torch.mm(q, T.t()), (q * q).sum(1), tn, k)
                knn_vote(labels[idx.long()], classes)

        def unfused():
            for s in range(0, nq, 4096):
                q = Q[s:s + 4096]
                d2 = torch.addmm((q * q).sum(1)[:, None] + tn[None, :], q, T.t(), alpha=-2.0)
                idx = torch.topk(torch.sqrt(torch.abs(d2)), k, dim=1, largest=False, sorted=True).indices
                knn_vote(labels[idx], classes)

        tf = timeit(fused, args.reps)
        ts = timeit(split, args.reps) if k <= ko.MAX_K and not args.only_fused else None
        tu = None if args.only_fused else timeit(unfused, args.reps)
        gemm_tflops = 2.0 * nq * n * d / tf / 1e12
        print(json.dumps({"bench": "KnnModel predict", "queries": nq, "train": n, "dim": d, "k": k,
                          "fused_ms": round(tf * 1e3, 2), "split_ms": None if ts is None else round(ts * 1e3, 2),
                          "torch_chain_ms": None if tu is None else round(tu * 1e3, 2),
                          "speedup_vs_torch": None if tu is None else round(tu / tf, 2),
                          "fused_kernel": ko.fused_supported(k, n, d, dev), "queries_per_s": round(nq / tf, 1),
                          "effective_fp32_tflops": round(gemm_tflops, 1)}), flush=True)
        del Q, T, labels, tn, pack
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
