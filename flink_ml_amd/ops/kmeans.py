"""Bindings for ``csrc/kmeans.hip`` plus the host reference (exact reference semantics, fp64).

``assign`` = findClosest for every row (K8); ``KMeansRound`` = one Lloyd step on the rank's
partition producing the all-reduce payload ``[k·D sums | k counts]`` (K9), deterministic.
"""
from __future__ import annotations

import math

import os

import numpy as np
import torch

from . import native
from .native import c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_kmeans_set_sched": [c_int],
    "fmlx_kmeans_assign_bf16": [c_void_p, c_long, c_long, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                c_void_p, c_void_p],
    "fmlx_kmeans_assign_generic": [c_int, c_void_p, c_long, c_long, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                   c_void_p],
    "fmlx_kmeans_chunk_sum": [c_int, c_void_p, c_long, c_int, c_void_p, c_void_p, c_void_p, c_int, c_long, c_void_p,
                              c_void_p],
    "fmlx_kmeans_cluster_sum": [c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "fmlx_kmeans_chunk_sum_bf16v": [c_void_p, c_long, c_int, c_void_p, c_void_p, c_void_p, c_int, c_long, c_void_p,
                                    c_void_p],
    "fmlx_kmeans_offsets": [c_void_p, c_long, c_int, c_void_p, c_void_p, c_void_p],
    "fmlx_sorted_bounds": [c_void_p, c_long, c_int, c_void_p, c_void_p],
    "fmlx_kmeans_finalize": [c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                             c_void_p],
    "fmlx_group_max_keys": [],
    "fmlx_group_by_key": [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "fmlx_group_stable_max_keys": [],
    "fmlx_group_stable_scratch": ([c_long, c_int], c_long),
    "fmlx_group_by_key_stable": [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
})

# rows grouped by cluster with the hand-written STABLE counting sort (csrc/groupsort.hip
# st_*: per-tile histograms, column scan, ordered scatter — rows of a cluster stay in row order,
# so the centroid sums are bit-reproducible) for k <= 2048; larger k takes the arrival-order
# counting sort (sums reproducible to rounding), or the stable radix sort of sort.hip when
# FMLX_DETERMINISTIC=1. GROUP_SORT=False forces the radix sort (A/B and tests).
GROUP_SORT = True
DETERMINISTIC = os.environ.get("FMLX_DETERMINISTIC", "0") == "1"

METRICS = {"euclidean": 0, "manhattan": 1, "cosine": 2}
CHUNK = 256
# (A split round — part p's grouping + gather-sum on a side stream under part p + 1's assign —
# measured 3.98-4.06 vs 3.77-3.86 ms/iter unsplit at the 12.5M x 128, k = 1024 shard and was removed
# in round 5: the assign fills every CU and the gather-sum beside it slows it more than it hides;
# profiles/r4/kmeans_assign_lds_split_ab.jsonl.)
MFMA_KS = (1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16)


def mfma_ks(D: int) -> int:
    """Padded number of 16-wide K steps for the MFMA assign kernel (0 if D is too wide)."""
    need = (D + 15) // 16
    for ks in MFMA_KS:
        if ks >= need:
            return ks
    return 0


# MFMA assign schedule (fmlx_kmeans_set_sched): 1 = the pipelined kernel for D = 64/128 (norms in
# the matrix core, LDS-DMA centroid ring, B fragments one tile ahead; other widths take the plain
# loop), 0 = the plain loop everywhere (A/B and tests). FMLX_KMEANS_SCHED overrides. 12.5M x 128,
# k = 1024 on one MI355X: 3.53 ms (plain) → 3.18 ms (pipelined); the other variants measured over
# rounds 2-4 were removed in round 5 (history in csrc/kmeans.hip).
ASSIGN_SCHED = int(os.environ.get("FMLX_KMEANS_SCHED", "1"))
_sched_applied = None


def set_assign_sched(mode: int) -> None:
    global _sched_applied
    native.call("fmlx_kmeans_set_sched", int(mode))
    _sched_applied = int(mode)


def mfma_ok(X: torch.Tensor, metric: str) -> bool:
    return (X.device.type == "cuda" and X.dtype == torch.bfloat16 and metric == "euclidean"
            and X.stride(1) == 1 and X.stride(0) % 2 == 0 and X.data_ptr() % 4 == 0 and mfma_ks(X.shape[1]) > 0)


class CentroidBuffers:
    """Device-side centroid representations consumed by the assign kernels."""

    def __init__(self, k: int, D: int, device, acc_dtype):
        self.k, self.D = k, D
        self.kpad = max(32, (k + 31) // 32 * 32)
        self.KS = mfma_ks(D) or (D + 15) // 16
        self.DP = self.KS * 16
        self.cent = torch.zeros((k, D), dtype=acc_dtype, device=device)
        self.cnorm = torch.zeros(k, dtype=acc_dtype, device=device)          # ‖c‖ (acc dtype)
        self.Cb = torch.zeros((self.kpad, self.DP), dtype=torch.bfloat16, device=device)
        self.cnorm_b = torch.full((self.kpad,), float("inf"), dtype=torch.float32, device=device)  # ‖c_bf16‖²
        # the pipelined MFMA assign's B_aug rows (‖c‖² split into three bf16s), rebuilt from
        # cnorm_b by every assign launch
        self.baug = torch.empty(self.kpad * 2, dtype=torch.int32, device=device)
        self.weights = torch.zeros(k, dtype=torch.float64, device=device)
        self._pack = None

    def set(self, centroids: torch.Tensor) -> None:
        # the k x D representations are formed on the host and copied over once (a fit's initial
        # centroids come from the host anyway): on the device the norm / pow / scatter ops would
        # each load their torch code object at first use, ~10-40 ms apiece in a fresh process
        c = torch.as_tensor(centroids).detach().to(device="cpu", dtype=self.cent.dtype)
        cb = c.to(torch.bfloat16)
        Cb = torch.zeros((self.kpad, self.DP), dtype=torch.bfloat16)
        Cb[: self.k, : self.D] = -2 * cb  # the MFMA assign consumes −2·c (exact in bf16)
        nb = torch.full((self.kpad,), float("inf"), dtype=torch.float32)
        nb[: self.k] = (cb.float() * cb.float()).sum(1)
        self.cent.copy_(c)
        self.cnorm.copy_(torch.linalg.vector_norm(c.to(torch.float64), dim=1).to(self.cent.dtype))
        self.Cb.copy_(Cb)
        self.cnorm_b.copy_(nb)
        self._pack = None

    def fp32_pack(self):
        """The current centroids as the fused KNN kernel's training pack (fp32). Refreshed in place
        on every call: the finalize kernel rewrites ``cent`` on the device, and inside a captured
        round the refresh replays with it."""
        c = self.cent.to(torch.float32)
        if self._pack is None:
            from . import knn as knn_ops

            self._pack = knn_ops.TrainPack(c, (c * c).sum(1))
        else:
            self._pack.refresh(c, (c * c).sum(1))
        return self._pack


# fp32 euclidean assign from GEMM_ASSIGN_MIN_ROWS rows: "fused" = the fused KNN kernel with k = 1
# (D <= 128; 1M x 100, k=10: 9.24 ms per 10-round fit vs 9.69 through the GEMM), "gemm" = library
# GEMM + argmin for few centroids; small inputs take the one-launch wave-per-row kernel (the
# fused path's pack refresh + merge launches cost more than they save there)
FP32_ASSIGN = os.environ.get("FMLX_KMEANS_FP32_ASSIGN", "fused")
GEMM_ASSIGN_MAX_K = 64       # fp32 euclidean assign through a library GEMM up to this many centroids
GEMM_ASSIGN_ROWS = 1 << 22   # rows per GEMM chunk (bounds the n×k distance block)
GEMM_ASSIGN_MIN_ROWS = 1 << 18  # below this the one-launch wave kernel wins (the GEMM path is ~6 launches)


def assign(X: torch.Tensor, cb: CentroidBuffers, metric: str, out: torch.Tensor = None) -> torch.Tensor:
    """Index of the closest centroid for every row (reference ``DistanceMeasure.findClosest``)."""
    n, D = X.shape
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=X.device)
    if n == 0:
        return out
    if X.device.type != "cuda":
        return torch_assign(X, cb.cent, metric).to(torch.int32)
    if mfma_ok(X, metric):
        if _sched_applied is None:
            set_assign_sched(ASSIGN_SCHED)
        native.call("fmlx_kmeans_assign_bf16", native.ptr(X), X.stride(0), n, D, cb.KS, native.ptr(cb.Cb),
                    native.ptr(cb.cnorm_b), cb.kpad, native.ptr(out), native.ptr(cb.baug), native.stream_ptr(X.device))
        return out
    if X.dtype not in (torch.float32, torch.float64):
        X = X.to(torch.float32)
    X = X if X.stride(1) == 1 else X.contiguous()
    if X.dtype == torch.float32 and metric == "euclidean" and FP32_ASSIGN == "fused" and n >= GEMM_ASSIGN_MIN_ROWS:
        from . import knn as knn_ops

        if knn_ops.fused_supported(1, cb.k, D, X.device):
            # the fused KNN kernel with k = 1: fp32 MFMA distances with the argmin in registers
            # (ties → lower centroid index, NaN never wins), no n×k block in HBM
            pack = cb.fp32_pack()
            out.copy_(knn_ops.fused_topk(X, pack, 1).view(-1))
            return out
    if X.dtype == torch.float32 and metric == "euclidean" and cb.k <= GEMM_ASSIGN_MAX_K and n >= GEMM_ASSIGN_MIN_ROWS:
        # few centroids: the distance "GEMM" X·Cᵀ is one bandwidth-bound library GEMM (fp32
        # accumulate) plus an n×k argmin; the wave-per-row kernel is latency-bound at this shape
        C = cb.cent.to(torch.float32)
        cn2 = (C * C).sum(1)
        for r0 in range(0, n, GEMM_ASSIGN_ROWS):
            Xc = X[r0:r0 + GEMM_ASSIGN_ROWS]
            # ‖c‖² − 2x·c: the per-row ‖x‖² does not move the argmin (no n×D temporary for it)
            d = torch.addmm(cn2.unsqueeze(0), Xc, C.t(), alpha=-2.0)
            d.nan_to_num_(nan=float("inf"))  # NaN distances never win, like torch_assign / the kernels
            out[r0:r0 + Xc.shape[0]] = torch.argmin(d, dim=1).to(torch.int32)  # first (lowest) index on ties
        return out
    C = cb.cent.to(X.dtype).contiguous()
    cn = cb.cnorm.to(X.dtype).contiguous()
    native.call("fmlx_kmeans_assign_generic", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), n, D,
                native.ptr(C), native.ptr(cn), cb.k, METRICS[metric], native.ptr(out), native.stream_ptr(X.device))
    return out


def torch_assign(X: torch.Tensor, C: torch.Tensor, metric: str) -> torch.Tensor:
    """Host reference of findClosest (EuclideanDistanceMeasure.java:53-73 incl. pruning order)."""
    X = X.to(torch.float64)
    C = C.to(device=X.device, dtype=torch.float64)
    if X.shape[0] == 0:
        return torch.zeros(0, dtype=torch.int64)
    if metric == "euclidean":
        pn = torch.linalg.vector_norm(X, dim=1)
        cn = torch.linalg.vector_norm(C, dim=1)
        d2 = torch.clamp(pn[:, None] * pn[:, None] + (cn * cn)[None, :] - 2.0 * (X @ C.T), min=0.0)
        d2 = torch.where(torch.isnan(d2), torch.full_like(d2, float("inf")), d2)
        return torch.argmin(d2, dim=1)  # argmin returns the first minimum: lowest index on ties
    if metric == "manhattan":
        d = torch.cdist(X, C, p=1)
    else:
        d = 1.0 - (X @ C.T) / torch.linalg.vector_norm(X, dim=1)[:, None] / torch.linalg.vector_norm(C, dim=1)[None, :]
    return torch.argmin(d, dim=1)


class KMeansRound:
    """One Lloyd iteration on a device-resident partition: assign → ordered chunk sums →
    per-cluster sums/counts. ``payload`` is the fixed-size all-reduce buffer."""

    def __init__(self, X: torch.Tensor, k: int, metric: str):
        self.X = X
        self.n, self.D = X.shape
        self.k = k
        self.metric = metric
        dev = X.device
        self.acc = torch.float64 if X.dtype == torch.float64 else torch.float32
        self.labels = torch.empty(self.n, dtype=torch.int32, device=dev)
        self.max_chunks = (self.n + CHUNK - 1) // CHUNK + k
        self.partial = torch.zeros((self.max_chunks, self.D), dtype=self.acc, device=dev)
        self.payload = torch.zeros(k * self.D + k, dtype=self.acc, device=dev)
        self.zero_i64 = torch.zeros(1, dtype=torch.int64, device=dev)
        self.fast = (dev.type == "cuda" and X.dtype == torch.bfloat16 and self.D in (8, 16, 32, 64, 128, 256, 512)
                     and X.stride(1) == 1 and X.stride(0) % 8 == 0 and X.data_ptr() % 16 == 0)
        lib = native.kernels() if dev.type == "cuda" else None
        self.stable = dev.type == "cuda" and GROUP_SORT and k <= lib.fmlx_group_stable_max_keys()
        self.group = (dev.type == "cuda" and GROUP_SORT and not self.stable and not DETERMINISTIC
                      and k <= lib.fmlx_group_max_keys())
        if dev.type == "cuda":
            self.offsets = torch.zeros(k + 1, dtype=torch.int64, device=dev)
            self.chunk_off = torch.zeros(k + 1, dtype=torch.int64, device=dev)
            self.order32 = torch.empty(self.n, dtype=torch.int32, device=dev)
        if self.stable:
            self.gscratch = torch.empty(max(1, int(lib.fmlx_group_stable_scratch(self.n, k))), dtype=torch.int32,
                                        device=dev)
        elif self.group:
            self.gcounts = torch.zeros(k, dtype=torch.int32, device=dev)  # re-zeroed by the scan kernel
            self.gcursor = torch.zeros(k, dtype=torch.int32, device=dev)
        if dev.type == "cuda" and not self.stable and not self.group:
            # more keys than the counting sort's LDS histograms hold: the stable segmented LSD radix
            # sort (radix.hip, one segment) over ceil(log2 k) bits, buffers allocated once
            from . import glm as _glm

            self.bits = max(1, int(k - 1).bit_length())
            self.iota = torch.arange(self.n, dtype=torch.int32, device=dev)
            self.sort_keys = torch.empty(self.n, dtype=torch.int32, device=dev)
            self.sort_vals = torch.empty(self.n, dtype=torch.int32, device=dev)
            self.sort_keys_alt = torch.empty(self.n, dtype=torch.int32, device=dev)
            self.sort_vals_alt = torch.empty(self.n, dtype=torch.int32, device=dev)
            self.sort_scratch = torch.empty(_glm.seg_sort_scratch([0, self.n], self.bits), dtype=torch.int32,
                                            device=dev)
            odd = _glm.seg_sort_passes(self.bits) & 1
            self.keys_sorted = self.sort_keys_alt if odd else self.sort_keys
            self.order32 = self.sort_vals_alt if odd else self.sort_vals

    def run(self, cb: CentroidBuffers) -> torch.Tensor:
        X = self.X
        if self.n == 0:
            self.payload.zero_()
            return self.payload
        assign(X, cb, self.metric, self.labels)
        stream = native.stream_ptr(X.device)
        if self.stable:
            # stable counting sort by cluster + cluster / chunk offsets (groupsort.hip st_*)
            native.call("fmlx_group_by_key_stable", native.ptr(self.labels), self.n, self.k, CHUNK,
                        native.ptr(self.gscratch), native.ptr(self.offsets), native.ptr(self.chunk_off),
                        native.ptr(self.order32), stream)
        elif self.group:
            # counting sort by cluster + cluster / chunk offsets, no library sort (groupsort.hip)
            native.call("fmlx_group_by_key", native.ptr(self.labels), self.n, self.k, CHUNK, native.ptr(self.gcounts),
                        native.ptr(self.gcursor), native.ptr(self.offsets), native.ptr(self.chunk_off),
                        native.ptr(self.order32), stream)
        else:
            from . import glm as _glm

            self.sort_keys.copy_(self.labels)
            self.sort_vals.copy_(self.iota)
            _glm.seg_sort(self.sort_keys, self.sort_vals, [0, self.n], [0], self.bits, self.sort_keys_alt,
                          self.sort_vals_alt, self.sort_scratch)
            # cluster boundaries on the device (no host sync: the round is hipGraph-capturable)
            native.call("fmlx_kmeans_offsets", native.ptr(self.keys_sorted), self.n, self.k, native.ptr(self.offsets),
                        native.ptr(self.chunk_off), stream)
        offsets, chunk_off = self.offsets, self.chunk_off
        if self.fast:
            native.call("fmlx_kmeans_chunk_sum_bf16v", native.ptr(X), X.stride(0), self.D, native.ptr(self.order32),
                        native.ptr(offsets), native.ptr(chunk_off), self.k, self.max_chunks, native.ptr(self.partial),
                        stream)
        else:
            order = self.order32.to(torch.int64)
            Xs = X if X.dtype in (torch.bfloat16, torch.float32, torch.float64) else X.to(torch.float32)
            native.call("fmlx_kmeans_chunk_sum", native.dtype_code(Xs.dtype), native.ptr(Xs), Xs.stride(0), self.D,
                        native.ptr(order), native.ptr(offsets), native.ptr(chunk_off), self.k, self.max_chunks,
                        native.ptr(self.partial), stream)
        native.call("fmlx_kmeans_cluster_sum", int(self.acc == torch.float64), native.ptr(self.partial), self.D,
                    native.ptr(offsets), native.ptr(chunk_off), self.k, native.ptr(self.payload),
                    native.stream_ptr(X.device))
        return self.payload

    def finalize(self, cb: CentroidBuffers, payload: torch.Tensor) -> None:
        native.call("fmlx_kmeans_finalize", int(self.acc == torch.float64), native.ptr(payload), self.D, self.k,
                    native.ptr(cb.cent), native.ptr(cb.weights), native.ptr(cb.Cb), cb.DP, native.ptr(cb.cnorm_b),
                    native.ptr(cb.cnorm), native.stream_ptr(self.X.device))


def torch_round_payload(X: torch.Tensor, C: torch.Tensor, metric: str) -> torch.Tensor:
    """Host reference for one round's [sums | counts] (CentroidsUpdateAccumulator, KMeans.java:269-300)."""
    k, D = C.shape
    X = X.to(torch.float64)
    out = torch.zeros(k * D + k, dtype=torch.float64)
    if X.shape[0] == 0:
        return out
    lab = torch_assign(X, C, metric)
    sums = torch.zeros((k, D), dtype=torch.float64).index_add_(0, lab, X)
    out[: k * D] = sums.reshape(-1)
    out[k * D:] = torch.bincount(lab, minlength=k).to(torch.float64)
    return out


def torch_finalize(payload: torch.Tensor, k: int, D: int):
    sums = payload[: k * D].reshape(k, D)
    counts = payload[k * D:]
    cent = sums * (1.0 / counts)[:, None]  # scal(1/count): 0 rows → NaN like the reference
    return cent, counts


def group_by_key(keys: torch.Tensor, k: int, chunk: int = 0, stable: bool = False):
    """Rows grouped by an int32 key in [0, k) on the device (csrc/groupsort.hip counting sort):
    returns (order int32 [m], offsets int64 [k + 1], chunk_off int64 [k + 1] or None), where
    ``order[offsets[c]:offsets[c+1]]`` are the rows with key c (in row order with ``stable``,
    k ≤ ``fmlx_group_stable_max_keys()``; otherwise in arrival order, k ≤ ``fmlx_group_max_keys()``)
    and m = offsets[k] (keys outside [0, k) are dropped)."""
    dev = keys.device
    n = keys.numel()
    keys = keys.to(torch.int32).contiguous()
    if stable:
        lib = native.kernels()
        scratch = torch.empty(max(1, int(lib.fmlx_group_stable_scratch(n, int(k)))), dtype=torch.int32, device=dev)
        offsets = torch.empty(k + 1, dtype=torch.int64, device=dev)
        chunk_off = torch.empty(k + 1, dtype=torch.int64, device=dev) if chunk > 0 else None
        order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        native.call("fmlx_group_by_key_stable", native.ptr(keys), n, int(k), int(chunk), native.ptr(scratch),
                    native.ptr(offsets), native.ptr(chunk_off), native.ptr(order), native.stream_ptr(dev))
        m = int(offsets[k].item())
        return order[:m], offsets, chunk_off
    counts = torch.zeros(k, dtype=torch.int32, device=dev)
    cursor = torch.empty(k, dtype=torch.int32, device=dev)
    offsets = torch.empty(k + 1, dtype=torch.int64, device=dev)
    chunk_off = torch.empty(k + 1, dtype=torch.int64, device=dev) if chunk > 0 else None
    order = torch.empty(n, dtype=torch.int32, device=dev)
    native.call("fmlx_group_by_key", native.ptr(keys), n, int(k), int(chunk), native.ptr(counts), native.ptr(cursor),
                native.ptr(offsets), native.ptr(chunk_off), native.ptr(order), native.stream_ptr(dev))
    m = int(offsets[k].item())
    return order[:m], offsets, chunk_off
