"""Exact distributed order statistics by radix select (replaces gathering the data for
RobustScaler / Imputer(median) quantiles).

Each value maps to an order-preserving signed integer key (IEEE bits, magnitude bits flipped for
negatives). The k-th smallest key of every column is found digit by digit from the most
significant end: per pass, one ``bincount`` of (column, digit) over the still-matching
candidates, an all-reduce of the [d, 2^b] histogram across ranks and a prefix scan that picks
the digit holding rank k. The data never leaves its rank; the cost is 64/b (fp64) or 32/b (fp32)
streaming passes over the shard plus d·2^b integers of communication per pass.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch

from ..parallel import comm
from . import native
from .native import c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_radix_hist": [c_int, c_void_p, c_long, c_long, c_int, c_void_p, c_int, c_int, c_int, c_long, c_void_p,
                        c_void_p, c_void_p],
})

_BITS = 11
_MAXQ = 4  # quantiles per kernel pass (LDS histogram [Q][16][256])
_M63 = 0x7FFFFFFFFFFFFFFF


def _keys(X: torch.Tensor):
    if X.dtype == torch.float64:
        b = X.contiguous().view(torch.int64)
        return torch.where(b < 0, b ^ _M63, b), 64
    b = X.to(torch.float32).contiguous().view(torch.int32).to(torch.int64)
    return torch.where(b < 0, b ^ 0x7FFFFFFF, b), 32


def _from_keys(sk: torch.Tensor, nbits: int, dtype) -> torch.Tensor:
    if nbits == 64:
        return torch.where(sk < 0, sk ^ _M63, sk).view(torch.float64).to(dtype)
    b = torch.where(sk < 0, sk ^ 0x7FFFFFFF, sk).to(torch.int32)
    return b.view(torch.float32).to(dtype)


def kth_smallest(X: torch.Tensor, k: torch.Tensor, valid: torch.Tensor = None, distributed: bool = False):
    """Per-column k-th smallest (1-based ranks ``k`` [d]; global over ranks when distributed) of
    X [n, d] among the entries where ``valid`` (default: not NaN)."""
    n, d = X.shape
    dev = X.device
    sk, nbits = _keys(X)
    cand = (~torch.isnan(X)) if valid is None else valid.clone()
    kk = k.to(dev, torch.int64).clone()
    col = torch.arange(d, device=dev, dtype=torch.int64)[None, :]
    passes, s = [], nbits
    while s > 0:
        b = min(_BITS, s)
        s -= b
        passes.append((s, b))
    sel_key = torch.zeros(d, dtype=torch.int64, device=dev)
    for i, (shift, b) in enumerate(passes):
        mask = (1 << b) - 1
        if i == 0:  # top digit carries the sign: bias it into [0, 2^b)
            digit = (sk >> shift) + (1 << (b - 1))
        else:
            digit = (sk >> shift) & mask
        bins = (col * (1 << b) + digit)[cand]
        hist = torch.bincount(bins, minlength=d * (1 << b)).reshape(d, 1 << b)
        if distributed:
            hist = comm.all_reduce_sum(hist)
        cum = torch.cumsum(hist, dim=1)
        sel = torch.clamp(torch.searchsorted(cum, kk[:, None]).reshape(d), max=mask)
        before = torch.where(sel > 0, cum.gather(1, torch.clamp(sel - 1, min=0)[:, None]).reshape(d),
                             torch.zeros_like(kk))
        kk = kk - before
        cand = cand & (digit == sel[None, :])
        part = (sel - (1 << (b - 1))) if i == 0 else sel
        sel_key = sel_key | (part << shift) if i else (part << shift)
    return _from_keys(sel_key, nbits, X.dtype)


def quantile_ranks(counts: torch.Tensor, ps: Sequence[float], rel_err: float):
    """1-based ranks under the reference QuantileSummary query semantics for each p
    (``QuantileSummary.java:237-364`` on exact data): p <= relErr -> the minimum, p >= 1 - relErr ->
    the maximum, otherwise rank ceil(p·n)."""
    out = []
    for p in ps:
        if p <= rel_err:
            out.append(torch.ones_like(counts))
        elif p >= 1 - rel_err:
            out.append(counts.clone())
        else:
            out.append(torch.clamp(torch.ceil(p * counts.to(torch.float64)).to(torch.int64), min=1))
    return out


def _unsigned_to_value(u: torch.Tensor, nbits: int) -> torch.Tensor:
    """Inverse of the kernel's order-preserving unsigned key (held as an int64 bit pattern)."""
    if nbits == 64:
        bits = torch.where(u < 0, u ^ torch.iinfo(torch.int64).min, ~u)
        return bits.view(torch.float64)
    top = u >= (1 << 31)
    bits = torch.where(top, u - (1 << 31), (~u) & 0xFFFFFFFF)
    bits = torch.where(bits >= (1 << 31), bits - (1 << 32), bits)
    return bits.to(torch.int32).view(torch.float32)


def kth_smallest_device(X: torch.Tensor, ks, distributed: bool = False, nq: int = 0) -> torch.Tensor:
    """k-th smallest (1-based ``ks`` [Q, d], Q <= 4) of every column of a GPU matrix, NaNs skipped,
    by the ``radixselect.hip`` histogram kernel: 4 (fp32) / 8 (fp64) passes of 8-bit digits for
    all Q ranks at once; per pass only the [Q, d, 256] histogram is all-reduced. ``ks`` may also be
    a function of the columns' (global) non-NaN counts — the top digit's histogram, which every
    rank target shares — returning the ranks (``nq`` of them): no separate counting pass."""
    if X.dtype not in (torch.float32, torch.float64):
        X = X.to(torch.float32)
    if X.stride(1) != 1:
        X = X.contiguous()
    n, d = X.shape
    rank_fn = ks if callable(ks) else None
    Q = nq if rank_fn is not None else ks.shape[0]
    assert 1 <= Q <= _MAXQ and (rank_fn is not None or ks.shape[1] == d)
    nbits = 64 if X.dtype == torch.float64 else 32
    dev = X.device
    groups = (d + 15) // 16
    chunks = int(max(1, min(256, (2048 + groups - 1) // groups, (n + 255) // 256)))
    while chunks > 1 and chunks * Q * d * 256 * 4 > (256 << 20):
        chunks //= 2
    part = torch.empty(chunks * Q * d * 256, dtype=torch.int32, device=dev)
    hist = torch.empty((Q, d, 256), dtype=torch.int64, device=dev)
    prefix = torch.zeros((Q, d), dtype=torch.int64, device=dev)
    # the per-pass digit choice runs on the host over the small [Q, d, 256] histogram (integer
    # exact; on the device its cumsum / searchsorted / gather kernels would each load a torch code
    # object at first use): one histogram copy down and one prefix copy up per pass
    prefix_h = torch.zeros((Q, d), dtype=torch.int64)
    kk = None if rank_fn is not None else ks.to(device="cpu", dtype=torch.int64).clone()
    for i, shift in enumerate(range(nbits - 8, -1, -8)):
        # the top digit's histogram is the same for every rank target: count it once
        q_eff = 1 if i == 0 else Q
        if i:
            prefix.copy_(prefix_h)
        native.call("fmlx_radix_hist", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), n, d,
                    native.ptr(prefix), q_eff, shift, int(i == 0), chunks, native.ptr(part), native.ptr(hist),
                    native.stream_ptr(dev))
        if i == 0:
            h = (comm.all_reduce_sum(hist[:1].contiguous()) if distributed else hist[:1]).cpu()
            if rank_fn is not None:
                kk = rank_fn(h[0].sum(-1)).to(device="cpu", dtype=torch.int64).clone()
                assert kk.shape == (Q, d)
            h = h.expand(Q, d, 256)
        else:
            h = (comm.all_reduce_sum(hist.contiguous()) if distributed else hist).cpu()
        cum = torch.cumsum(h, dim=2)
        sel = torch.clamp(torch.searchsorted(cum, kk[..., None]).squeeze(-1), max=255)
        before = torch.where(sel > 0, cum.gather(2, torch.clamp(sel - 1, min=0)[..., None]).squeeze(-1),
                             torch.zeros_like(kk))
        kk = kk - before
        prefix_h = (prefix_h << 8) | sel
    return _unsigned_to_value(prefix_h, nbits).to(dev)


def column_quantiles(X: torch.Tensor, ps: Sequence[float], rel_err: float, distributed: bool = False) -> torch.Tensor:
    """[len(ps), d] quantiles of every column (NaNs ignored), exact and rank-local."""
    if X.device.type == "cuda" and 0 < len(ps) <= _MAXQ and X.dim() == 2 and X.shape[1] > 0:
        # the non-NaN counts come from the select's first (top-digit) histogram
        def ranks_of(counts):
            if bool((counts == 0).any()):
                raise RuntimeError("Cannot query percentiles without any records inserted.")
            return torch.stack(quantile_ranks(counts, ps, rel_err))

        return kth_smallest_device(X, ranks_of, distributed, nq=len(ps)).to(torch.float64)
    valid = ~torch.isnan(X)
    counts = valid.sum(0).to(torch.int64)
    if distributed:
        counts = comm.all_reduce_sum(counts)
    if bool((counts == 0).any()):
        raise RuntimeError("Cannot query percentiles without any records inserted.")
    ranks = quantile_ranks(counts, ps, rel_err)
    if X.device.type == "cuda":
        out = []
        for j in range(0, len(ranks), _MAXQ):
            out.append(kth_smallest_device(X, torch.stack(ranks[j:j + _MAXQ]), distributed).to(torch.float64))
        return torch.cat(out)
    return torch.stack([kth_smallest(X, r, valid, distributed).to(torch.float64) for r in ranks])
