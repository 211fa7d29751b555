"""Bindings for ``csrc/knn.hip``: KNN predict's distance epilogue + per-query top-k (K13).

``topk_from_products(G, qn, tn, k)`` takes the fp32 product block ``G = Q·Tᵀ`` (one hipBLASLt GEMM)
and returns the indices of the k nearest training points per query, nearest first, ties to the
lower index — ``KnnModel.predictLabel`` (reference ``KnnModel.java:154-194``) semantics.
"""
from __future__ import annotations

import os

import torch

from . import native
from .native import c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_knn_topk": [c_void_p, c_long, c_long, c_long, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                      c_void_p, c_void_p, c_void_p],
})

MAX_K = 32
# KnnModel routes k above this to the sort path: the per-lane insertion lists get long enough that
# insertions, not HBM, bound the scan (measured: k=32 is ~5x slower than addmm+topk; k<=16 is
# 2-3.4x faster — README "KNN")
ROUTE_MAX_K = 16
# G block budget (bytes): large enough to amortise the per-block GEMM/vote launches, small
# enough to bound the transient memory
G_BLOCK_BYTES = 512 << 20


def supported(k: int, n: int, device) -> bool:
    return torch.device(device).type == "cuda" and 1 <= k <= MAX_K and k <= n < 2 ** 31 - 1


def query_block(n: int) -> int:
    b = G_BLOCK_BYTES // max(1, 4 * n)
    return int(min(16384, max(1024, b // 4 * 4)))


# waves wanted per launch and the shortest column segment worth a wave. Few, long segments win:
# every segment pays ~k·ln(L/k) insertions before its bound settles (sweep on MI355X: 2048 waves
# beat 4096/8192/16384 by 10-60%)
TARGET_WAVES = int(os.environ.get("FMLX_KNN_WAVES", "2048"))
MIN_SEGMENT = 2048


def segments(nq: int, n: int) -> int:
    """Column segments per query row so a launch has enough waves in flight."""
    want = -(-TARGET_WAVES // max(1, nq))
    return int(max(1, min(want, n // MIN_SEGMENT, 256)))


def topk_from_products(G: torch.Tensor, qn: torch.Tensor, tn: torch.Tensor, k: int, with_dist: bool = False):
    """k nearest columns of every row of ``G`` under ``sqrt(|qn_r + tn_c − 2·G_rc|)``."""
    nq, n = G.shape
    if not (G.dtype == torch.float32 and qn.dtype == torch.float32 and tn.dtype == torch.float32):
        raise TypeError("knn top-k expects fp32 products and norms")
    if G.stride(1) != 1 or qn.numel() != nq or tn.numel() != n or not supported(k, n, G.device):
        raise ValueError("knn top-k: bad shapes G=%s qn=%s tn=%s k=%d" % (tuple(G.shape), tuple(qn.shape),
                                                                         tuple(tn.shape), k))
    qn, tn = qn.contiguous(), tn.contiguous()
    idx = torch.empty((nq, k), dtype=torch.int32, device=G.device)
    dist = torch.empty((nq, k), dtype=torch.float32, device=G.device) if with_dist else None
    S = segments(nq, n)
    ws_d = torch.empty(nq * S * k, dtype=torch.float32, device=G.device) if S > 1 else None
    ws_i = torch.empty(nq * S * k, dtype=torch.int32, device=G.device) if S > 1 else None
    native.call("fmlx_knn_topk", native.ptr(G), G.stride(0), nq, n, S, native.ptr(qn), native.ptr(tn), k,
                native.ptr(idx), native.ptr(dist), native.ptr(ws_d), native.ptr(ws_i), native.stream_ptr(G.device))
    return (idx, dist) if with_dist else idx
