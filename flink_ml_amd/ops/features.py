"""Device ops shared by the feature transformers (``csrc/colstats.hip``) with torch fallbacks on CPU.

``column_stats`` is the K15 single-pass column reduction (sum, Σx², min, max) and
``affine_cols`` the K16 fused per-column ``(x - sub) * mul + add``; both work on the rank's
partition and the estimators all-reduce the fixed-size statistics across ranks.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import native
from .native import c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_colstats": [c_int, c_void_p, c_long, c_long, c_int, c_void_p, c_int, c_void_p, c_void_p],
    "fmlx_affine_cols": [c_int, c_int, c_void_p, c_long, c_long, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p],
})


def column_stats(X: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Per-column sum, sumsq, min, max (fp64) of a dense [n, d] tensor on the rank."""
    n, d = X.shape
    dev = X.device
    if n == 0:
        inf = float("inf")
        return {"sum": torch.zeros(d, dtype=torch.float64, device=dev),
                "sumsq": torch.zeros(d, dtype=torch.float64, device=dev),
                "min": torch.full((d,), inf, dtype=torch.float64, device=dev),
                "max": torch.full((d,), -inf, dtype=torch.float64, device=dev), "count": 0}
    if dev.type == "cuda" and X.dtype in (torch.float32, torch.float64, torch.bfloat16) and X.stride(1) == 1:
        nb = max(1, min(1024, (n + 1023) // 1024))
        part = torch.empty((nb, 4, d), dtype=torch.float64, device=dev)
        res = torch.empty((4, d), dtype=torch.float64, device=dev)
        native.call("fmlx_colstats", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), n, d, native.ptr(part),
                    nb, native.ptr(res), native.stream_ptr(dev))
        return {"sum": res[0], "sumsq": res[1], "min": res[2], "max": res[3], "count": n}
    Xd = X.to(torch.float64)
    return {"sum": Xd.sum(0), "sumsq": (Xd * Xd).sum(0), "min": Xd.min(0).values, "max": Xd.max(0).values,
            "count": n}


def affine_cols(X: torch.Tensor, sub: Optional[torch.Tensor] = None, mul: Optional[torch.Tensor] = None,
                add: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``(x - sub) * mul + add`` per column; output fp64 on CPU, fp32/fp64 on GPU."""
    n, d = X.shape
    dev = X.device
    prep = lambda v: None if v is None else v.to(device=dev, dtype=torch.float64).contiguous()  # noqa: E731
    sub, mul, add = prep(sub), prep(mul), prep(add)
    if dev.type == "cuda" and X.dtype in (torch.float32, torch.float64, torch.bfloat16) and X.stride(1) == 1:
        out_dt = torch.float64 if X.dtype == torch.float64 else torch.float32
        out = torch.empty((n, d), dtype=out_dt, device=dev)
        if n:
            native.call("fmlx_affine_cols", native.dtype_code(X.dtype), native.dtype_code(out_dt), native.ptr(X),
                        X.stride(0), n, d, native.ptr(sub), native.ptr(mul), native.ptr(add), native.ptr(out),
                        native.stream_ptr(dev))
        return out
    out = X.to(torch.float64)
    if sub is not None:
        out = out - sub
    if mul is not None:
        out = out * mul
    if add is not None:
        out = out + add
    return out


native.register_kernel_sigs({
    "fmlx_group_colstats": [c_int, c_void_p, c_long, c_long, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int,
                            c_void_p, c_void_p],
})

MAX_GROUPS = 32


def group_colstats(X: torch.Tensor, gidx: Optional[torch.Tensor] = None, G: int = 1,
                   w: Optional[torch.Tensor] = None):
    """Per-group weighted column sums S[G, d] = Σ_{group(r)=g} w_r·x_r, plus Σx and Σx² (all fp64)
    in one pass (``csrc/groupstats.hip`` on the GPU, G <= 32)."""
    n, d = X.shape
    dev = X.device
    if (dev.type == "cuda" and 1 <= G <= MAX_GROUPS and X.dtype in (torch.float32, torch.float64, torch.bfloat16)
            and X.stride(1) == 1 and n > 0):
        nb = max(1, min(1024, (n + 2047) // 2048))
        part = torch.empty((nb, (G + 2) * d), dtype=torch.float64, device=dev)
        res = torch.empty(((G + 2) * d,), dtype=torch.float64, device=dev)
        g = gidx.to(device=dev, dtype=torch.int32).contiguous() if gidx is not None else None
        ww = w.to(device=dev, dtype=torch.float64).contiguous() if w is not None else None
        native.call("fmlx_group_colstats", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), n, d, native.ptr(g),
                    G, native.ptr(ww), native.ptr(part), nb, native.ptr(res), native.stream_ptr(dev))
        return res[:G * d].reshape(G, d), res[G * d:(G + 1) * d], res[(G + 1) * d:]
    Xd = X.to(torch.float64)
    wx = Xd * w.to(dev, torch.float64)[:, None] if w is not None else Xd
    if gidx is None:
        S = wx.sum(0, keepdim=True).expand(G, d).clone() if G == 1 else None
    else:
        S = torch.zeros((G, d), dtype=torch.float64, device=dev).index_add_(0, gidx.to(dev).long(), wx)
    return S, Xd.sum(0), (Xd * Xd).sum(0)
