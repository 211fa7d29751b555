"""Bindings for ``csrc/knn.hip``: KNN predict's distances + per-query top-k (K13).

Two device paths, both with ``KnnModel.predictLabel`` (reference ``KnnModel.java:154-194``)
semantics — the k nearest training points per query, nearest first, ties to the lower index:

* ``fused_topk(Q, pack, k)`` (D ≤ 128, k ≤ 64): ONE kernel computes the distances on the fp32
  matrix cores and keeps the top-k in registers; the nq×n distance block never reaches HBM.
  ``TrainPack`` is the training matrix pre-arranged once per model for the kernel's tile copy.
* ``topk_from_products(G, qn, tn, k)`` (any D, k ≤ 32): takes an fp32 product block
  ``G = Q·Tᵀ`` from a library GEMM and scans it once (the fallback for D > 128).
"""
from __future__ import annotations

import os

import torch

from . import native
from .native import c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_knn_topk": [c_void_p, c_long, c_long, c_long, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                      c_void_p, c_void_p, c_void_p],
    "fmlx_knn_fused": [c_void_p, c_long, c_long, c_int, c_void_p, c_long, c_int, c_int, c_int, c_void_p, c_void_p,
                       c_void_p, c_void_p, c_void_p],
    "fmlx_knn_fused_blocks_per_cu": [c_int, c_int],
})

FUSED_MAX_K = 64
FUSED_MAX_D = 128
# the shortest training segment worth a block (in 64-row tiles) and the most segments tried
FUSED_MIN_TILES = 16
FUSED_MAX_SEGMENTS = 64
_SLOTS = {}


def _slots(k: int, dp: int, device) -> int:
    """Fused-kernel blocks resident at once on the device (occupancy × CUs)."""
    key = (k, dp, str(device))
    if key not in _SLOTS:
        per_cu = native.kernels().fmlx_knn_fused_blocks_per_cu(k, dp)
        _SLOTS[key] = max(1, per_cu) * torch.cuda.get_device_properties(device).multi_processor_count
    return _SLOTS[key]


def fused_supported(k: int, n: int, d: int, device) -> bool:
    return (torch.device(device).type == "cuda" and 1 <= k <= FUSED_MAX_K and k <= n < 2 ** 31 - 128
            and 1 <= d <= FUSED_MAX_D)


class TrainPack:
    """Training points as the fused kernel's LDS image, one block of floats per 64-row tile
    (built once per model, on the device): ``[sub 2][h 2][r 32][dp + 4]`` with
    ``T[64·t + 32·sub + r][2·s + h]`` at ``s`` (zero padded: D to 2·dp, dp = ceil(D/2) rounded up
    to 4, and 4 pad columns that keep the kernel's LDS reads conflict-free), then the tile's 64
    squared norms in a 256-float block, so the kernel stages a tile with plain 1-KiB LDS-DMA copies."""

    def __init__(self, T: torch.Tensor, tnorm: torch.Tensor):
        n, d = T.shape
        self.n, self.d = int(n), int(d)
        self.dp = -(-(-(-d // 2)) // 4) * 4
        self.nt = -(-n // 64)
        dev = T.device
        self.Tt = torch.zeros((self.nt, 128 * (self.dp + 4) + 256), dtype=torch.float32, device=dev)
        self._Tp = torch.zeros((self.nt * 64, 2 * self.dp), dtype=torch.float32, device=dev)
        self._tn = torch.zeros(self.nt * 64, dtype=torch.float32, device=dev)
        self.refresh(T, tnorm)

    def refresh(self, T: torch.Tensor, tnorm: torch.Tensor) -> "TrainPack":
        """Re-fills the pack in place from new values of the same shape (device copies only, so
        it can run inside a captured graph — KMeans re-packs its centroids every round)."""
        nt, dp, n, d = self.nt, self.dp, self.n, self.d
        self._Tp[:n, :d].copy_(T)
        rows = self.Tt[:, :128 * (dp + 4)].view(nt, 2, 2, 32, dp + 4)
        rows[..., :dp].copy_(self._Tp.view(nt, 2, 32, dp, 2).permute(0, 1, 4, 2, 3))
        self._tn[:n].copy_(tnorm)
        self.Tt[:, 128 * (dp + 4):128 * (dp + 4) + 64].copy_(self._tn.view(nt, 64))
        return self


def fused_segments(nq: int, n: int, k: int, slots: int) -> int:
    """Training segments per query block. Cost model in tile units: the blocks run in
    ceil(blocks / slots) rounds of (tiles per segment + a list fill of ~1 + k/16 tiles); a bad
    split strands a mostly empty last round (782 query blocks × 2 segments on 512 slots ran 4
    rounds for 3.05 rounds of work), so every S up to the cap is scored and the cheapest wins."""
    bq = -(-nq // 128)
    nt = -(-n // 64)
    smax = int(max(1, min(FUSED_MAX_SEGMENTS, nt // FUSED_MIN_TILES, 256)))
    fill = 1.0 + k / 16.0
    best, best_cost = 1, None
    for S in range(1, smax + 1):
        cost = -(-(bq * S) // slots) * (-(-nt // S) + fill)
        if best_cost is None or cost < best_cost * 0.995:
            best, best_cost = S, cost
    return best


def fused_topk(Q: torch.Tensor, pack: "TrainPack", k: int, with_dist: bool = False, segments: int = 0):
    """k nearest training points of every row of ``Q`` [nq, D] (fp32) in one fused kernel."""
    nq, d = Q.shape
    if Q.dtype != torch.float32 or d != pack.d or not fused_supported(k, pack.n, d, Q.device):
        raise ValueError("knn fused: bad inputs Q=%s %s, D=%d, n=%d, k=%d" % (tuple(Q.shape), Q.dtype, pack.d,
                                                                              pack.n, k))
    if Q.stride(1) != 1:
        Q = Q.contiguous()
    S = int(segments) or fused_segments(nq, pack.n, k, _slots(k, pack.dp, Q.device))
    idx = torch.empty((nq, k), dtype=torch.int32, device=Q.device)
    dist = torch.empty((nq, k), dtype=torch.float32, device=Q.device) if with_dist else None
    ws_d = torch.empty(nq * S * k, dtype=torch.float32, device=Q.device) if S > 1 else None
    ws_i = torch.empty(nq * S * k, dtype=torch.int32, device=Q.device) if S > 1 else None
    native.call("fmlx_knn_fused", native.ptr(Q), Q.stride(0), nq, d, native.ptr(pack.Tt), pack.n, pack.dp, k, S,
                native.ptr(idx), native.ptr(dist), native.ptr(ws_d), native.ptr(ws_i), native.stream_ptr(Q.device))
    return (idx, dist) if with_dist else idx

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


# ---- any k, fp32 or fp64: radix selection over a library-GEMM product block (csrc/knn_select.hip)
native.register_kernel_sigs({
    "fmlx_knn_select": [c_int, c_void_p, c_long, c_long, c_long, c_void_p, c_void_p, c_int, c_void_p, c_long,
                        c_void_p],
})
SELECT_MAX_K = 8192  # csrc/knn_select.hip SEL_KMAX (the k winners are sorted in LDS)
SELECT_BLOCK_BYTES = 1 << 30


def select_supported(k: int, n: int, dtype, device) -> bool:
    return (torch.device(device).type == "cuda" and dtype in (torch.float32, torch.float64)
            and 1 <= k <= SELECT_MAX_K and k <= n < 2 ** 31 - 1)


def select_query_block(n: int, es: int) -> int:
    """Queries per product block: the [block, n] block within SELECT_BLOCK_BYTES."""
    return int(max(1, min(1 << 16, SELECT_BLOCK_BYTES // max(1, es * n))))


def select_topk(G: torch.Tensor, qn: torch.Tensor, tn: torch.Tensor, k: int) -> torch.Tensor:
    """int32 [nq, k]: the k nearest columns of every row of ``G`` under ``|qn_r + tn_c − 2·G_rc|``,
    nearest first, ties to the lower column (``KnnModel.java:154-194``) — any k up to
    SELECT_MAX_K, fp32 or fp64 (one 1024-thread block per row: radix passes, then a sort of the k)."""
    nq, n = G.shape
    dt = G.dtype
    if dt not in (torch.float32, torch.float64) or qn.dtype != dt or tn.dtype != dt:
        raise TypeError("knn select expects fp32 or fp64 products and norms of one dtype")
    if G.stride(1) != 1 or qn.numel() != nq or tn.numel() != n or not select_supported(k, n, dt, G.device):
        raise ValueError("knn select: bad shapes G=%s qn=%s tn=%s k=%d" % (tuple(G.shape), tuple(qn.shape),
                                                                          tuple(tn.shape), k))
    qn, tn = qn.contiguous(), tn.contiguous()
    idx = torch.empty((nq, k), dtype=torch.int32, device=G.device)
    if nq:
        native.call("fmlx_knn_select", int(dt == torch.float64), native.ptr(G), G.stride(0), nq, n, native.ptr(qn),
                    native.ptr(tn), int(k), native.ptr(idx), k, native.stream_ptr(G.device))
    return idx
