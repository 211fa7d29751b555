"""Device sorts and the BinaryClassificationEvaluator kernels (``csrc/radix.hip``,
``csrc/binclass.hip``): stable LSD radix sorts of 64-bit keys with 32-bit payloads, over only the
key bits that differ (an OR/AND reduction of the keys picks the range), and the evaluator's
sorted-order scans. No library sort is involved."""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np
import torch

from . import native
from .native import c_double, c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_sort_bits_scratch": ([c_void_p, c_int, c_int], c_long),
    "fmlx_sort_u64": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_long,
                      c_void_p],
    "fmlx_bc_tile": [],
    "fmlx_bc_keys": [c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_void_p],
    "fmlx_bc_metrics": [c_void_p, c_void_p, c_void_p, c_long, c_double, c_double, c_double, c_double,
                        c_void_p, c_void_p, c_void_p, c_void_p],
})

U64 = torch.int64  # uint64 keys live in int64 storage (bit patterns; never compared by torch)


def bit_range(orand: torch.Tensor) -> Tuple[int, int]:
    """[lo, hi) of the key bits that differ between keys with this {OR, AND} (0, 0: all equal)."""
    o, a = (int(v) & ((1 << 64) - 1) for v in orand.cpu().tolist())
    diff = o ^ a
    if diff == 0:
        return 0, 0
    lo = (diff & -diff).bit_length() - 1
    return lo, diff.bit_length()


def sort_u64(keys: torch.Tensor, vals: torch.Tensor, bounds: Sequence[int], bit_lo: int,
             bit_hi: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Stable sort of (uint64 key, uint32 payload) pairs inside every segment ``[bounds[s],
    bounds[s+1])`` by key bits [bit_lo, bit_hi) (≤ 32 segments). Returns (keys, vals) sorted (the
    inputs are used as ping-pong buffers)."""
    if bit_hi <= bit_lo or keys.numel() == 0:
        return keys, vals
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.int64))
    S = len(b) - 1
    lib = native.kernels()
    need = int(lib.fmlx_sort_bits_scratch(b.ctypes.data, S, bit_hi - bit_lo))
    if need < 0:
        raise ValueError("sort_u64: bad segment table (S=%d, bits=%d)" % (S, bit_hi - bit_lo))
    scratch = torch.empty(max(1, need), dtype=torch.int32, device=keys.device)
    ka, va = torch.empty_like(keys), torch.empty_like(vals)
    rc = lib.fmlx_sort_u64(native.ptr(keys), native.ptr(vals), native.ptr(ka), native.ptr(va), b.ctypes.data, S,
                           int(bit_lo), int(bit_hi), native.ptr(scratch), scratch.numel(),
                           native.stream_ptr(keys.device))
    if rc < 0 or rc > 1:
        raise RuntimeError("fmlx_sort_u64 failed: %d" % rc)
    return (ka, va) if rc == 1 else (keys, vals)


def _u8(pos: torch.Tensor) -> torch.Tensor:
    return pos.contiguous().view(torch.uint8) if pos.dtype == torch.bool else pos.to(torch.uint8).contiguous()


def sort_scores_desc(score: torch.Tensor, pos: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(keys, payloads) of fp64 ``score`` in descending order (Double.compare of −score: NaN last,
    −0 tied with +0), stable: equal scores keep their row order. Payload = row id | label << 31
    (``pos``: the rows' labels, bool)."""
    n = score.numel()
    dev = score.device
    if n >= 1 << 31:
        raise ValueError("at most 2^31 - 1 rows per rank")
    keys = torch.empty(n, dtype=U64, device=dev)
    rows = torch.empty(n, dtype=torch.int32, device=dev)
    orand = torch.tensor([0, -1], dtype=U64, device=dev)
    native.call("fmlx_bc_keys", native.ptr(score), native.ptr(_u8(pos)), n, native.ptr(keys), native.ptr(rows),
                native.ptr(orand), native.stream_ptr(dev))
    lo, hi = bit_range(orand)
    return sort_u64(keys, rows, [0, n], lo, hi)


def binary_metrics(keys: torch.Tensor, rows: torch.Tensor, w, before_t: float, before_f: float,
                   tot_t: float, tot_f: float) -> torch.Tensor:
    """[Σ_pos w·(gs + ge), Σ_pos w, Σ_neg w, lorenz, pr, ks] over the sorted rows (fp64, device);
    ``rows``: the payloads of ``sort_scores_desc``; ``w``: weights by original row, or None."""
    n = keys.numel()
    dev = keys.device
    tile = int(native.kernels().fmlx_bc_tile())
    nt = max(1, -(-n // tile))
    scratch = torch.empty(8 * nt, dtype=torch.int64, device=dev)
    part = torch.empty(6 * nt, dtype=torch.float64, device=dev)
    out = torch.empty(6, dtype=torch.float64, device=dev)
    w = None if w is None else w.to(torch.float64).contiguous()
    native.call("fmlx_bc_metrics", native.ptr(keys), native.ptr(rows), native.ptr(w), n,
                float(before_t), float(before_f), float(tot_t), float(tot_f), native.ptr(scratch), native.ptr(part),
                native.ptr(out), native.stream_ptr(dev))
    return out
