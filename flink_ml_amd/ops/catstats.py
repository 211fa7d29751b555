"""Device contingency statistics (``csrc/catstats.hip``): sorted distinct values, label indices
and (feature, value, label) counts for NaiveBayes (K22) and ChiSqTest (K20), with no library
sort / unique / bincount. Integer-valued columns with a small value range (the categorical
case) are counted straight into an LDS-privatised table; anything else goes through the stable
64-bit radix sort of each column (``ops/sorting.py``) and a distinct-id scan.

All functions take CUDA tensors; the CPU reference of every result is the torch code in
``models/stats.py`` / ``models/naive_bayes.py``.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np
import torch

from . import native, sorting
from .native import c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_cs_tile": [],
    "fmlx_cs_lds_ints": [],
    "fmlx_cs_flags": [c_int, c_void_p, c_long, c_long, c_int, c_void_p, c_void_p, c_void_p],
    "fmlx_cs_ihist": [c_int, c_void_p, c_long, c_long, c_int, c_long, c_int, c_void_p, c_void_p],
    "fmlx_cs_hist": [c_int, c_void_p, c_long, c_long, c_int, c_void_p, c_int, c_long, c_int, c_void_p, c_void_p],
    "fmlx_cs_col_keys": [c_int, c_void_p, c_long, c_long, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "fmlx_cs_distinct": [c_void_p, c_void_p, c_long, c_int, c_int, c_void_p, c_long, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p],
    "fmlx_cs_chist": [c_void_p, c_long, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "fmlx_cs_small_distinct": [c_void_p, c_long, c_long, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                               c_void_p],
})

# integer tables up to this many cells are counted directly (value range × labels × features)
MAX_TABLE = 1 << 27
# integer labels / values are histogrammed directly up to this range
MAX_INT_RANGE = 1 << 24
SORT_SEGMENTS = 32  # columns per segmented sort call (radix.hip RS_MAXS)


def _mat(X: torch.Tensor) -> torch.Tensor:
    if X.dim() == 1:
        X = X.reshape(-1, 1)
    if X.dtype not in (torch.float32, torch.float64):
        X = X.to(torch.float64)
    if X.stride(1) != 1:
        X = X.contiguous()
    return X


def flags(X: torch.Tensor) -> Tuple[float, float, bool]:
    """(min, max, any non-integer or non-finite) of all elements of X (device reduction)."""
    X = _mat(X)
    n, d = X.shape
    if n * d == 0:
        return float("inf"), float("-inf"), False
    dev = X.device
    part = torch.empty(3 * 1024, dtype=torch.float64, device=dev)
    out = torch.empty(3, dtype=torch.float64, device=dev)
    native.call("fmlx_cs_flags", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), n, d, native.ptr(part),
                native.ptr(out), native.stream_ptr(dev))
    mn, mx, non = out.cpu().tolist()
    return mn, mx, non != 0.0


native.register_kernel_sigs({
    "fmlx_cv_tfdf": [c_void_p, c_void_p, c_long, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
})
CODE_COUNTS_MAX_V = 4096  # dictionary sizes of the one-pass count kernel (csrc/hash.hip cv_tfdf_kernel)
CODE_COUNTS_SEG = 4096  # codes per pseudo-document (the kernel's unit of work per wave)


def code_counts_first(codes: torch.Tensor, V: int):
    """(count, first position) per dictionary code in [0, V) of a device int32 code column, host
    int64 arrays, in one pass of the CountVectorizer tf kernel over fixed-size segments (the
    column cut into pseudo-documents; their document frequencies are not used). None when V is
    beyond the kernel's LDS tables."""
    n = codes.shape[0]
    if not codes.is_cuda or V < 1 or V > CODE_COUNTS_MAX_V or n >= (1 << 32):
        return None
    dev = codes.device
    codes = codes.to(torch.int32).contiguous()
    seg = CODE_COUNTS_SEG
    nd = max(1, -(-n // seg))
    off = torch.from_numpy(np.minimum(np.arange(nd + 1, dtype=np.int64) * seg, n)).to(dev)
    out = torch.zeros(3 * V, dtype=torch.int64, device=dev)  # count | (unused) | first
    out[2 * V:] = n
    if n:
        native.call("fmlx_cv_tfdf", native.ptr(codes), native.ptr(off), nd, V, native.ptr(out), native.ptr(out[V:]),
                    native.ptr(out[2 * V:]), native.stream_ptr(dev))
    h = out.cpu().numpy().reshape(3, V)
    return h[0], h[2]


SMALL_DISTINCT_TABLE_MAX = 2048  # LDS hash-set slots (csrc/catstats.hip small_distinct_kernel)


def bounded_distinct_counts(X: torch.Tensor, cap: int):
    """Per column of a device fp64 matrix: the number of distinct values (NaN one value, −0 == +0)
    when it is at most ``cap``, else cap + 1 — one early-exit hash-set pass (a continuous column
    stops after a few hundred rows). None when cap is too large for the LDS table."""
    X = _mat(X)
    if X.dtype != torch.float64:
        X = X.to(torch.float64)
    if X.stride(1) != 1:
        X = X.contiguous()
    n, d = X.shape
    S = 1
    while S < 2 * cap + 256:
        S <<= 1
    if cap < 1 or S > SMALL_DISTINCT_TABLE_MAX or d > 65535:
        return None
    dev = X.device
    gtab = torch.full((d * S,), -1, dtype=torch.int64, device=dev)
    ints = torch.zeros(2 * d, dtype=torch.int32, device=dev)  # counts | overflow flags
    if n and d:
        native.call("fmlx_cs_small_distinct", native.ptr(X), X.stride(0), n, d, int(cap), S, native.ptr(gtab),
                    native.ptr(ints), native.ptr(ints[d:]), native.stream_ptr(dev))
    h = ints.cpu().numpy()
    return np.where(h[d:] != 0, cap + 1, h[:d]).astype(np.int64)


def int_hist(v: torch.Tensor, lo: int, R: int) -> torch.Tensor:
    """int32 counts of the integer values lo … lo + R − 1 of the 1-D tensor ``v`` (device)."""
    dev = v.device
    if v.dtype not in (torch.float32, torch.float64, torch.int32):
        v = v.to(torch.float64)
    v = v.reshape(-1, 1).contiguous()
    counts = torch.zeros(max(1, R), dtype=torch.int32, device=dev)
    if v.shape[0]:
        native.call("fmlx_cs_ihist", native.dtype_code(v.dtype), native.ptr(v), 1, v.shape[0], 0, int(lo), int(R),
                    native.ptr(counts), native.stream_ptr(dev))
    return counts[:R]


def distinct_codes(X: torch.Tensor) -> Tuple[torch.Tensor, List[torch.Tensor]]:
    """Per column j of X [n, d]: the sorted distinct values (fp64, device; −0 folded into +0, NaN
    last) and every row's index into them: codes int32 [d, n]."""
    X = _mat(X)
    n, d = X.shape
    dev = X.device
    codes = torch.empty((d, n), dtype=torch.int32, device=dev)
    vals: List[torch.Tensor] = []
    tile = int(native.kernels().fmlx_cs_tile())
    for j0 in range(0, d, SORT_SEGMENTS):
        nc = min(SORT_SEGMENTS, d - j0)
        m = n * nc
        keys = torch.empty(m, dtype=torch.int64, device=dev)
        rows = torch.empty(m, dtype=torch.int32, device=dev)
        orand = torch.tensor([0, -1], dtype=torch.int64, device=dev)
        native.call("fmlx_cs_col_keys", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), n, j0, nc,
                    native.ptr(keys), native.ptr(rows), native.ptr(orand), native.stream_ptr(dev))
        lo, hi = sorting.bit_range(orand)
        keys, rows = sorting.sort_u64(keys, rows, [c * n for c in range(nc + 1)], lo, hi)
        nt = max(1, -(-m // tile))
        tcnt = torch.empty(nt + 1, dtype=torch.int64, device=dev)
        uval = torch.empty(max(1, m), dtype=torch.float64, device=dev)
        ucol = torch.empty(max(1, m), dtype=torch.int32, device=dev)
        colfirst = torch.zeros(nc, dtype=torch.int64, device=dev)
        native.call("fmlx_cs_distinct", native.ptr(keys), native.ptr(rows), n, nc, j0, native.ptr(tcnt), 0,
                    native.ptr(codes[j0:j0 + nc]), native.ptr(uval), native.ptr(ucol), native.ptr(colfirst),
                    native.stream_ptr(dev))
        if n == 0:
            vals += [torch.empty(0, dtype=torch.float64, device=dev) for _ in range(nc)]
            continue
        first = colfirst.cpu().tolist() + [int(tcnt[nt].item())]
        vals += [uval[first[c]:first[c + 1]] for c in range(nc)]
    return codes, vals


def sorted_unique(v: torch.Tensor) -> torch.Tensor:
    """Sorted distinct values of a 1-D tensor (fp64): a presence histogram for small-range
    integers, else the sorted-column distinct pass."""
    v = v.reshape(-1)
    if v.numel() == 0:
        return torch.empty(0, dtype=torch.float64, device=v.device)
    mn, mx, non = flags(v)
    if not non and mx - mn + 1 <= MAX_INT_RANGE:
        cnt = int_hist(v, int(mn), int(mx - mn) + 1)
        present = np.nonzero(cnt.cpu().numpy())[0]
        return torch.as_tensor(present + int(mn), dtype=torch.float64).to(v.device)
    return distinct_codes(v)[1][0]


def label_index(y: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """int32 index of every y in the sorted ``labels`` (a binary search per row)."""
    return torch.searchsorted(labels.to(torch.float64), y.reshape(-1).to(torch.float64)).to(torch.int32)


def label_counts(li: torch.Tensor, L: int) -> torch.Tensor:
    """int64 rows per label index 0 … L − 1."""
    return int_hist(li.to(torch.int32), 0, L).to(torch.int64)


def int_table(X: torch.Tensor, li: torch.Tensor, L: int, vmin: int, V: int) -> torch.Tensor:
    """int32 [d, L, V] counts of the integer values vmin … vmin + V − 1 per (feature, label
    index) — one pass over X (LDS-privatised table when d·L·V fits)."""
    X = _mat(X)
    n, d = X.shape
    dev = X.device
    counts = torch.zeros(max(1, d * L * V), dtype=torch.int32, device=dev)
    if n and d:
        native.call("fmlx_cs_hist", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), n, d,
                    native.ptr(li.to(torch.int32).contiguous()), L, int(vmin), int(V), native.ptr(counts),
                    native.stream_ptr(dev))
    return counts[:d * L * V].reshape(d, L, V)


def value_label_counts(X: torch.Tensor, li: torch.Tensor, L: int,
                       int_range: Optional[Tuple[float, float]] = None):
    """(feature, distinct value, label) counts of one rank's rows.

    Returns (counts int64 [d, L, Vmax] numpy, per-feature sorted distinct values as numpy fp64,
    per-feature slots of those values in the last axis). ``int_range`` = (min, max) when X is
    known to hold integers (the caller's flags, possibly all-reduced): the direct table path."""
    X = _mat(X)
    n, d = X.shape
    dev = X.device
    li = li.to(torch.int32).contiguous()
    if int_range is None:
        mn, mx, non = flags(X)
        int_range = None if non else (mn, mx)
    if int_range is not None and n and (int_range[1] - int_range[0] + 1) * L * d <= MAX_TABLE:
        vmin = int(int_range[0])
        V = int(int_range[1]) - vmin + 1
        c = int_table(X, li, L, vmin, V).cpu().numpy().astype(np.int64)
        present = c.sum(1) > 0
        slots = [np.nonzero(present[j])[0] for j in range(d)]
        return c, [(sl + vmin).astype(np.float64) for sl in slots], slots
    codes, vals = distinct_codes(X)
    Vn = [int(v.numel()) for v in vals]
    Vmax = max([1] + Vn)
    coloff = torch.arange(d, dtype=torch.int64, device=dev) * Vmax
    counts = torch.zeros(max(1, d * Vmax * L), dtype=torch.int32, device=dev)
    native.call("fmlx_cs_chist", native.ptr(codes), n, d, native.ptr(coloff), native.ptr(li), L, native.ptr(counts),
                native.stream_ptr(dev))
    c = counts[:d * Vmax * L].reshape(d, Vmax, L).permute(0, 2, 1).cpu().numpy().astype(np.int64)
    return c, [v.cpu().numpy() for v in vals], [np.arange(V) for V in Vn]


def global_value_label_counts(X: torch.Tensor, li: torch.Tensor, L: int):
    """(feature, distinct value, label) counts over ALL ranks on the native kernels — the keyed
    count of ``ChiSqTest.java:127-155`` / ``NaiveBayes.java:95-103`` without a keyed shuffle:

    * integer features whose [d, L, V] table (value range from the all-reduced min / max) has at
      most MAX_TABLE cells: one ``int_table`` pass per rank, then ONE all-reduce of the dense table;
    * otherwise every rank takes its per-column sorted distinct values (``value_label_counts``:
      radix sort + distinct pass), the ranks' value lists are all-gathered (padded to the longest,
      the padding repeating a real value of the column) and their union per column is one more
      ``distinct_codes`` pass; each rank places its local counts at their union slots (a host
      binary search over the small per-column lists) and one all-reduce sums the tables.

    Returns (counts float64 [d, L, Vmax] numpy, per-feature sorted distinct values (numpy fp64),
    per-feature slots of those values in the last axis) — the shape ``value_label_counts`` returns
    on one rank."""
    from ..parallel import comm

    X = _mat(X)
    n, d = X.shape
    dev = X.device
    mn, mx, non = flags(X) if n else (float("inf"), float("-inf"), False)
    f = comm.all_reduce(torch.tensor([-mn, mx, float(non)], dtype=torch.float64, device=dev), "max").tolist()
    mn, mx, non = -f[0], f[1], f[2] != 0.0
    if not non and mx >= mn and (mx - mn + 1) * L * d <= MAX_TABLE:
        vmin, V = int(mn), int(mx - mn) + 1
        cnt = comm.all_reduce_sum(int_table(X, li, L, vmin, V).to(torch.float64)) if n else \
            comm.all_reduce_sum(torch.zeros((d, L, V), dtype=torch.float64, device=dev))
        counts = cnt.cpu().numpy()
        present = counts.sum(1) > 0
        slots = [np.nonzero(present[j])[0] for j in range(d)]
        return counts, [(sl + vmin).astype(np.float64) for sl in slots], slots
    if n:
        c_loc, vals_loc, slots_loc = value_label_counts(X, li, L, int_range=None)
    else:
        c_loc, vals_loc, slots_loc = np.zeros((d, L, 1), np.int64), [np.zeros(0)] * d, [np.zeros(0, np.int64)] * d
    vl = np.array([len(v) for v in vals_loc], dtype=np.int64)
    M = int(comm.all_reduce(torch.tensor([int(vl.max()) if d else 0], dtype=torch.int64, device=dev), "max")[0])
    M = max(M, 1)
    pad = np.zeros((M, d), dtype=np.float64)
    for j in range(d):
        if vl[j]:
            pad[:vl[j], j] = vals_loc[j]
    # (the gathered blocks carry each rank's list lengths in a last row)
    blk = torch.from_numpy(np.concatenate([pad, vl[None, :].astype(np.float64)], 0)).to(dev)
    gathered = comm.all_gather_tensor(blk)
    G = torch.stack(gathered)                   # [world, M + 1, d]
    lens = G[:, M, :].cpu().numpy().astype(np.int64)  # [world, d]
    vals_g = G[:, :M, :]
    rows = torch.arange(M, device=dev)[None, :, None]
    valid = rows < torch.as_tensor(lens, device=dev)[:, None, :]
    # padding repeats a real value of its column (the first one of the first rank holding one)
    first_r = np.argmax(lens > 0, axis=0)
    fill = vals_g[torch.as_tensor(first_r, device=dev), 0, torch.arange(d, device=dev)]
    U = torch.where(valid, vals_g, fill[None, None, :]).reshape(-1, d)
    _, union = distinct_codes(U)
    union = [u.cpu().numpy() if int(lens[:, j].sum()) else np.zeros(0) for j, u in enumerate(union)]
    Umax = max([1] + [len(u) for u in union])
    T = np.zeros((d, L, Umax), dtype=np.float64)
    for j in range(d):
        if vl[j]:
            pos = np.searchsorted(union[j], vals_loc[j])
            T[j][:, pos] = c_loc[j][:, slots_loc[j]]
    T = comm.all_reduce_sum(torch.from_numpy(T).to(dev)).cpu().numpy()
    return T, union, [np.arange(len(u)) for u in union]
