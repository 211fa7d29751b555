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

_BITS = 11
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


def column_quantiles(X: torch.Tensor, ps: Sequence[float], rel_err: float, distributed: bool = False) -> torch.Tensor:
    """[len(ps), d] quantiles of every column (NaNs ignored), exact and rank-local."""
    valid = ~torch.isnan(X)
    counts = valid.sum(0).to(torch.int64)
    if distributed:
        counts = comm.all_reduce_sum(counts)
    if bool((counts == 0).any()):
        raise RuntimeError("Cannot query percentiles without any records inserted.")
    return torch.stack([kth_smallest(X, r, valid, distributed).to(torch.float64)
                        for r in quantile_ranks(counts, ps, rel_err)])
