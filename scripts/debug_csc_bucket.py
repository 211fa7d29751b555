#!/usr/bin/env python3
"""Diagnostics for radix.hip fmlx_csc_sort_split: runs it on a small run of batches and compares
pass 1 (keys_alt: stable by the high column bits), the column pointers and the row / value
payloads against numpy, printing where they first differ."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.ops import glm as gk, native  # noqa: E402


def main(d=3000, lens=(20_000, 0, 7_001, 30_000), seed=0):
    rng = np.random.default_rng(seed)
    S = len(lens)
    bound = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    m = int(bound[-1])
    cols = np.concatenate([np.sort(rng.integers(0, d, L)) if L else np.zeros(0, np.int64) for L in lens])
    rng.shuffle(cols)  # any order: the sort must keep it for equal columns
    slot = np.repeat(np.arange(S), lens)
    keys = (slot * d + cols).astype(np.int32)
    rows = rng.integers(0, 1 << 20, m).astype(np.int64)
    vbits = rng.integers(0, 1 << 31, m).astype(np.int64)
    pay = (vbits << 32) | rows
    bits = (d - 1).bit_length()
    dev = torch.device("cuda")
    k = torch.from_numpy(keys).to(dev)
    p = torch.from_numpy(pay).to(dev)
    k2, p2 = torch.empty_like(k), torch.empty_like(p)
    sc = torch.empty(gk.seg_sort_scratch(list(bound), bits), dtype=torch.int32, device=dev)
    off = 5
    erow = torch.full((m + off,), -7, dtype=torch.int32, device=dev)
    evals = torch.full((m + off,), -7, dtype=torch.int32, device=dev)
    b0 = 1
    colptr = torch.full((S + 2, d + 1), -9, dtype=torch.int32, device=dev)
    kb = np.ascontiguousarray((np.arange(S) * d).astype(np.int32))
    rc = native.kernels().fmlx_csc_sort_split(native.ptr(k), native.ptr(p), native.ptr(k2), native.ptr(p2),
                                              bound.ctypes.data, kb.ctypes.data, S, bits, d, native.ptr(sc),
                                              sc.numel(), native.ptr(erow), native.ptr(evals), off,
                                              native.ptr(colptr), b0, 0, native.stream_ptr(dev))
    torch.cuda.synchronize()
    print("rc", rc, "bits", bits)
    # pass 1 reference: per segment stable by high bits (key - kbase) >> 10
    ref_k2 = np.empty_like(keys)
    ref_p2 = np.empty_like(pay)
    order = np.empty(m, dtype=np.int64)
    for s in range(S):
        a, b = bound[s], bound[s + 1]
        o = np.argsort((keys[a:b] - s * d) >> 10, kind="stable")
        ref_k2[a:b] = keys[a:b][o]
        ref_p2[a:b] = pay[a:b][o]
        o2 = np.argsort(keys[a:b] - s * d, kind="stable")
        order[a:b] = a + o2
    gk2 = k2.cpu().numpy()
    gp2 = p2.cpu().numpy()
    bad = np.nonzero(gk2 != ref_k2)[0]
    print("pass1 keys mismatches", len(bad), bad[:10])
    bad = np.nonzero(gp2 != ref_p2)[0]
    print("pass1 payload mismatches", len(bad), bad[:10])
    er = erow.cpu().numpy()
    ev = evals.cpu().numpy()
    exp_rows = (pay[order] & 0xFFFFFFFF).astype(np.int32)
    exp_vals = (pay[order] >> 32).astype(np.int32)
    bad = np.nonzero(er[off:] != exp_rows)[0]
    print("erow mismatches", len(bad), bad[:10], "head", er[:off])
    bad = np.nonzero(ev[off:] != exp_vals)[0]
    print("evals mismatches", len(bad), bad[:10])
    cp = colptr.cpu().numpy()
    for s in range(S):
        a, b = bound[s], bound[s + 1]
        c = np.sort(keys[a:b] - s * d)
        exp = np.searchsorted(c, np.arange(d + 1)).astype(np.int32)
        exp[d] = b - a
        badc = np.nonzero(cp[b0 + s] != exp)[0]
        print("seg", s, "len", b - a, "colptr mismatches", len(badc), badc[:10],
              cp[b0 + s][badc[:5]] if len(badc) else "", exp[badc[:5]] if len(badc) else "")
    print("untouched rows", (cp[0] != -9).sum(), (cp[S + 1] != -9).sum())


if __name__ == "__main__":
    main()
    main(d=1_000_000, lens=(100_000, 3, 50_000), seed=1)
