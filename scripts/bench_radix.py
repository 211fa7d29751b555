#!/usr/bin/env python3
"""Segmented radix sort (csrc/radix.hip) at the sparse-SVC transpose shape: a run of ``--segs``
batches of ``--seg-len`` entries, keys = slot·d + column (d = 1M → 20 key bits), 64-bit
(value bits, row) payloads, split output on the last pass — µs per sort for each digit width,
interleaved repetitions (cdna_hip_programming.md §5.4 rule 24). One JSON line per width.
Usage: python scripts/bench_radix.py --bits 10,7 --reps 5"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.ops import glm as gk  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=10)
    ap.add_argument("--seg-len", type=int, default=6_400_000)
    ap.add_argument("--dim", type=int, default=1_000_000)
    ap.add_argument("--bits", default="10,7")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    S, L, d = a.segs, a.seg_len, a.dim
    n = S * L
    bounds = [s * L for s in range(S + 1)]
    kbase = [s * d for s in range(S)]
    keys = (torch.randint(0, d, (S, L), generator=g, device=dev, dtype=torch.int32)
            + torch.arange(S, device=dev, dtype=torch.int32)[:, None] * d).reshape(-1)
    pay = torch.randint(0, 1 << 62, (n,), generator=g, device=dev, dtype=torch.int64)
    kin = torch.empty_like(keys)
    pin = torch.empty_like(pay)
    kalt = torch.empty_like(keys)
    palt = torch.empty_like(pay)
    lo = torch.empty(n, dtype=torch.int32, device=dev)
    hi = torch.empty(n, dtype=torch.float32, device=dev)
    key_bits = (d - 1).bit_length()
    widths = [int(x) for x in a.bits.split(",")]
    res = {w: [] for w in widths}
    ref = None
    for rep in range(a.reps + 1):
        for w in widths:
            gk.SEG_SORT_DIGIT_BITS = w
            sc = torch.empty(gk.seg_sort_scratch(bounds, key_bits), dtype=torch.int32, device=dev)
            tot = 0.0
            for _ in range(a.iters):
                kin.copy_(keys)
                pin.copy_(pay)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ko, _ = gk.seg_sort(kin, pin, bounds, kbase, key_bits, kalt, palt, sc, split=(lo, hi, 0))
                torch.cuda.synchronize()
                tot += time.perf_counter() - t0
            if rep == 0:  # warm-up rep doubles as the cross-width exactness check
                cur = (ko.clone(), lo.clone(), hi.view(torch.int32).clone())
                if ref is None:
                    ref = cur
                else:
                    assert all(torch.equal(x, y) for x, y in zip(ref, cur)), "digit widths disagree"
                continue
            res[w].append(tot / a.iters * 1e6)
    for w, v in res.items():
        med = statistics.median(v)
        print(json.dumps({"digit_bits": w, "passes": gk.seg_sort_passes(key_bits) if w == 10 else -(-key_bits // w),
                          "pairs": n, "us_per_sort_median": round(med, 1), "us_min": round(min(v), 1),
                          "GB_per_s_per_pass_rw": round(n * 24 / (med / 1e6) / 1e9 /
                                                        (-(-key_bits // w)), 1)}), flush=True)


if __name__ == "__main__":
    main()
