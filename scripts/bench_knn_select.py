#!/usr/bin/env python3
"""KNN predict beyond the fused kernel (k > 64, fp64 parity mode): the select kernel
(ops/csrc/knn_select.hip) after the library GEMM vs torch.topk on the same distance block.
One JSON line per shape: ms of GEMM + select, of GEMM + addmm/abs + topk, and whether the
indices agree (exactly on integer data)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / reps, out


def main():
    from flink_ml_amd.ops import knn as ko
    from flink_ml_amd.ops import native

    native.kernels()
    dev = torch.device("cuda")
    for nq, n, d, k, dt in [(10_000, 100_000, 100, 128, torch.float32), (10_000, 100_000, 100, 1000, torch.float32),
                            (10_000, 100_000, 100, 10, torch.float64), (10_000, 100_000, 100, 500, torch.float64),
                            (2_000, 1_000_000, 64, 256, torch.float32)]:
        g = torch.Generator(device=dev).manual_seed(1)
        if "--float" in sys.argv:  # continuous data: few ties, the two-pass selection applies
            Q = torch.randn((nq, d), generator=g, device=dev, dtype=dt)
            T = torch.randn((n, d), generator=g, device=dev, dtype=dt)
        else:  # small integers: exact distances, many ties
            Q = torch.randint(-3, 4, (nq, d), generator=g, device=dev).to(dt)
            T = torch.randint(-3, 4, (n, d), generator=g, device=dev).to(dt)
        qn, tn = (Q * Q).sum(1), (T * T).sum(1)
        qb = ko.select_query_block(n, Q.element_size())

        def ours():
            out = []
            for s in range(0, nq, qb):
                q = Q[s:s + qb]
                out.append(ko.select_topk(torch.mm(q, T.t()), qn[s:s + qb], tn, k))
            return torch.cat(out)

        def lib():
            out = []
            for s in range(0, nq, qb):
                q = Q[s:s + qb]
                d2 = torch.addmm(qn[s:s + qb, None] + tn[None, :], q, T.t(), alpha=-2.0).abs_()
                out.append(torch.topk(d2, k, dim=1, largest=False, sorted=True).indices)
            return torch.cat(out)

        t_ours, a = timeit(ours)
        t_lib, b = timeit(lib)
        # topk does not promise the lower index among ties: compare the selected distances
        same = None
        if nq * n <= 2 ** 30:
            D = (qn[:, None] + tn[None, :] - 2 * Q @ T.t()).abs()
            same = bool(torch.equal(torch.gather(D, 1, a.long()), torch.gather(D, 1, b.long())))
            del D
        print(json.dumps({"data": "float" if "--float" in sys.argv else "int", "nq": nq, "n": n, "d": d, "k": k,
                          "dtype": str(dt).split(".")[-1],
                          "select_ms": round(t_ours, 3), "torch_topk_ms": round(t_lib, 3),
                          "same_distances": same}), flush=True)


if __name__ == "__main__":
    main()
