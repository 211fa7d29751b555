"""Device BLAS over columns of vectors (``csrc/blas.hip``).

The reference's ``linalg/BLAS.java:30-204`` works on one vector per call inside per-row map
functions. Here each op takes a whole column — dense rows ``X [n, d]`` (bf16 / fp32 / fp64) or a
``SparseColumn`` (CSR) — and runs as one HIP launch on the GPU; on CPU-only hosts the same
functions run the torch reference (fp64). Reductions accumulate in fp32 for bf16/fp32 rows and
fp64 for fp64 rows.

===========================  ========================================================
``BLAS.java``                here (batched over rows)
===========================  ========================================================
``dot(x, y)``                ``row_dot(X, Y)`` (dense·dense, CSR·CSR sorted merge),
                             ``gemv(X, v)`` (rows · one dense vector: dense or CSR)
``asum`` / ``norm2`` /       ``row_norm(X, p)`` (p = 1, 2, inf or any p ≥ 1)
``norm(p)``
``scal`` / ``axpy``          ``axpby(alpha, X, beta, Y)`` (scalar or per-row coefficients),
                             ``csr_axpy_dense`` (sparse x into dense rows, first k columns)
``hDot``                     ``hdot(v, X)`` (dense or CSR rows ∘ one vector)
``gemv(…, trans)``           ``gemv`` (N) / ``gemv_t(X, m)`` (Xᵀ·m, deterministic column sums)
(Normalizer map)             ``normalize(X, p)`` (norm + scale fused, one pass per row)
===========================  ========================================================
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional, Sequence

import torch

from ..table import SparseColumn
from . import native
from .native import c_double, c_int, c_long, c_void_p

native.register_kernel_sigs({
    "fmlx_blas_rowreduce": [c_int, c_int, c_void_p, c_long, c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_double,
                            c_void_p, c_void_p],
    "fmlx_blas_normalize": [c_int, c_int, c_void_p, c_long, c_long, c_int, c_double, c_int, c_void_p, c_long, c_void_p],
    "fmlx_blas_axpby": [c_int, c_void_p, c_long, c_void_p, c_long, c_long, c_int, c_double, c_void_p, c_double,
                        c_void_p, c_void_p],
    "fmlx_blas_hdot": [c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_void_p, c_long, c_void_p],
    "fmlx_blas_gemv_t_blocks": ([c_long], c_long),
    "fmlx_blas_gemv_t": [c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_void_p, c_void_p, c_double, c_void_p],
    "fmlx_blas_csr_rowreduce": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int, c_double,
                                c_void_p, c_void_p],
    "fmlx_blas_csr_scale": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p],
    "fmlx_blas_csr_axpy_dense": [c_int, c_void_p, c_void_p, c_void_p, c_double, c_long, c_int, c_void_p, c_long,
                                 c_void_p],
    "fmlx_blas_csr_csr_dot": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_void_p,
                              c_void_p],
    "fmlx_blas_gather_cols": [c_int, c_void_p, c_long, c_void_p, c_long, c_int, c_void_p, c_void_p],
    "fmlx_blas_gather_prod": [c_int, c_void_p, c_long, c_int, c_void_p, c_int, c_long, c_int, c_void_p, c_void_p],
    "fmlx_blas_interaction": [c_int, c_void_p, c_void_p, c_void_p, c_long, c_void_p, c_void_p],
})

OP_DOT, OP_DOTV, OP_NORM2, OP_NORM1, OP_NORMINF, OP_NORMP, OP_ASUM = range(7)


def _acc(dtype: torch.dtype) -> torch.dtype:
    return torch.float64 if dtype == torch.float64 else torch.float32


def _tpr(width: float) -> int:
    """Lanes per row: about 4 elements per lane, power of two in [4, 64]."""
    for t in (4, 8, 16, 32):
        if width <= 4 * t:
            return t
    return 64


def _dense_ok(X: torch.Tensor) -> bool:
    return X.is_cuda and X.dim() == 2 and X.stride(1) == 1 and X.dtype in (torch.float32, torch.float64,
                                                                           torch.bfloat16)


def _rowmajor(X: torch.Tensor) -> torch.Tensor:
    if X.dtype not in (torch.float32, torch.float64, torch.bfloat16):
        X = X.to(torch.float64)
    return X if X.stride(1) == 1 else X.contiguous()


def _csr_dev(X: SparseColumn):
    ip = X.indptr.to(torch.int64).contiguous()
    ix = X.indices.to(torch.int32).contiguous()
    v = X.values if X.values.dtype in (torch.float32, torch.float64) else X.values.to(torch.float64)
    return ip, ix, v.contiguous()


# ---------------------------------------------------------------------------------------------
# reductions
# ---------------------------------------------------------------------------------------------
def row_norm(X, p: float = 2.0) -> torch.Tensor:
    """‖row‖_p for every row (``BLAS.norm`` / ``norm2`` / ``asum`` for p = 1)."""
    if p < 1.0:
        raise ValueError("p value must >= 1.0, but the current p is : %s" % p)
    op = OP_NORMINF if math.isinf(p) else OP_NORM2 if p == 2.0 else OP_NORM1 if p == 1.0 else OP_NORMP
    if isinstance(X, SparseColumn):
        n = len(X)
        if X.values.is_cuda and n:
            ip, ix, v = _csr_dev(X)
            out = torch.empty(n, dtype=_acc(v.dtype), device=v.device)
            native.call("fmlx_blas_csr_rowreduce", native.dtype_code(v.dtype), _tpr(v.numel() / max(n, 1)),
                        native.ptr(ip), native.ptr(ix), native.ptr(v), None, n, op, float(p), native.ptr(out),
                        native.stream_ptr(v.device))
            return out
        rows = torch.repeat_interleave(torch.arange(n, device=X.values.device), X.indptr[1:] - X.indptr[:-1])
        a = X.values.to(torch.float64).abs()
        if math.isinf(p):
            return torch.zeros(n, dtype=torch.float64, device=a.device).scatter_reduce(0, rows, a, "amax")
        return torch.zeros(n, dtype=torch.float64, device=a.device).index_add_(0, rows, a ** p) ** (1.0 / p)
    X = _rowmajor(X)
    n, d = X.shape
    if _dense_ok(X) and n:
        out = torch.empty(n, dtype=_acc(X.dtype), device=X.device)
        native.call("fmlx_blas_rowreduce", native.dtype_code(X.dtype), _tpr(d), native.ptr(X), X.stride(0), None, 0,
                    None, n, d, op, float(p), native.ptr(out), native.stream_ptr(X.device))
        return out
    return torch.linalg.vector_norm(X.to(torch.float64), ord=p, dim=1)


def row_asum(X) -> torch.Tensor:
    return row_norm(X, 1.0)


def row_dot(X, Y) -> torch.Tensor:
    """Row-wise ``BLAS.dot`` of two equally shaped columns (dense·dense or CSR·CSR; CSR indices
    sorted within rows, as SparseVector keeps them)."""
    if isinstance(X, SparseColumn) != isinstance(Y, SparseColumn):
        raise TypeError("row_dot: mix a dense and a sparse column through gemv-like hdot instead")
    if isinstance(X, SparseColumn):
        n = len(X)
        if len(Y) != n or X.size != Y.size:
            raise ValueError("Vector size mismatched.")
        if X.values.is_cuda and n:
            ap, ai, av = _csr_dev(X)
            bp, bi, bv = _csr_dev(Y)
            bv = bv.to(av.dtype)
            out = torch.empty(n, dtype=_acc(av.dtype), device=av.device)
            native.call("fmlx_blas_csr_csr_dot", native.dtype_code(av.dtype), native.ptr(ap), native.ptr(ai),
                        native.ptr(av), native.ptr(bp), native.ptr(bi), native.ptr(bv), n, native.ptr(out),
                        native.stream_ptr(av.device))
            return out
        return (X.to_dense(torch.float64) * Y.to_dense(torch.float64)).sum(1)
    X, Y = _rowmajor(X), _rowmajor(Y)
    if X.shape != Y.shape:
        raise ValueError("Vector size mismatched.")
    n, d = X.shape
    if _dense_ok(X) and n:
        Y = Y.to(X.dtype)
        Y = Y if Y.stride(1) == 1 else Y.contiguous()
        out = torch.empty(n, dtype=_acc(X.dtype), device=X.device)
        native.call("fmlx_blas_rowreduce", native.dtype_code(X.dtype), _tpr(d), native.ptr(X), X.stride(0),
                    native.ptr(Y), Y.stride(0), None, n, d, OP_DOT, 2.0, native.ptr(out), native.stream_ptr(X.device))
        return out
    return (X.to(torch.float64) * Y.to(torch.float64)).sum(1)


def gemv(X, v) -> torch.Tensor:
    """y[r] = row_r · v (``BLAS.gemv`` 'N' with the rows as the matrix; dense or CSR rows)."""
    v = torch.as_tensor(v)
    if isinstance(X, SparseColumn):
        n = len(X)
        if X.values.is_cuda and n:
            ip, ix, vals = _csr_dev(X)
            vd = v.to(device=vals.device, dtype=torch.float64).contiguous()
            out = torch.empty(n, dtype=_acc(vals.dtype), device=vals.device)
            native.call("fmlx_blas_csr_rowreduce", native.dtype_code(vals.dtype), _tpr(vals.numel() / max(n, 1)),
                        native.ptr(ip), native.ptr(ix), native.ptr(vals), native.ptr(vd), n, OP_DOTV, 2.0,
                        native.ptr(out), native.stream_ptr(vals.device))
            return out
        rows = torch.repeat_interleave(torch.arange(n, device=X.values.device), X.indptr[1:] - X.indptr[:-1])
        vd = v.to(device=X.values.device, dtype=torch.float64)
        return torch.zeros(n, dtype=torch.float64, device=vd.device).index_add_(
            0, rows, X.values.to(torch.float64) * vd[X.indices.long()])
    X = _rowmajor(X)
    n, d = X.shape
    if _dense_ok(X) and n:
        vv = v.to(device=X.device, dtype=X.dtype).contiguous()
        out = torch.empty(n, dtype=_acc(X.dtype), device=X.device)
        native.call("fmlx_blas_rowreduce", native.dtype_code(X.dtype), _tpr(d), native.ptr(X), X.stride(0), None, 0,
                    native.ptr(vv), n, d, OP_DOTV, 2.0, native.ptr(out), native.stream_ptr(X.device))
        return out
    return X.to(torch.float64) @ v.to(device=X.device, dtype=torch.float64)


def gemv_t(X: torch.Tensor, m, y: Optional[torch.Tensor] = None, beta: float = 0.0) -> torch.Tensor:
    """y = Xᵀ·m (+ beta·y): ``BLAS.gemv`` with ``transMatrix``; fp64 result, fixed-order
    (deterministic) column sums."""
    X = _rowmajor(X)
    n, d = X.shape
    m = torch.as_tensor(m).to(device=X.device, dtype=torch.float64).contiguous()
    if y is None:
        y = torch.zeros(d, dtype=torch.float64, device=X.device)
        beta = 0.0
    if _dense_ok(X):
        nb = int(native.kernels().fmlx_blas_gemv_t_blocks(n))
        part = torch.empty((nb, d), dtype=_acc(X.dtype), device=X.device)
        native.call("fmlx_blas_gemv_t", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), native.ptr(m), n, d,
                    native.ptr(part), native.ptr(y), float(beta), native.stream_ptr(X.device))
        return y
    r = X.to(torch.float64).t() @ m
    if beta == 0.0:
        y.copy_(r)
    else:
        y.mul_(beta).add_(r)
    return y


# ---------------------------------------------------------------------------------------------
# element-wise
# ---------------------------------------------------------------------------------------------
def normalize(X, p: float = 2.0):
    """Every row scaled by 1/‖row‖_p (Normalizer; ``BLAS.norm`` + ``BLAS.scal``), norm and scale
    fused in one pass on the device."""
    if p < 1.0:
        raise ValueError("p value must >= 1.0, but the current p is : %s" % p)
    if isinstance(X, SparseColumn):
        norm = row_norm(X, p).to(torch.float64)
        return csr_scale(X, row_scale=1.0 / norm)
    X = _rowmajor(X)
    n, d = X.shape
    if _dense_ok(X) and n:
        out = torch.empty((n, d), dtype=_acc(X.dtype), device=X.device)
        native.call("fmlx_blas_normalize", native.dtype_code(X.dtype), _tpr(d), native.ptr(X), X.stride(0), n, d,
                    0.0 if math.isinf(p) else float(p), int(math.isinf(p)), native.ptr(out), out.stride(0),
                    native.stream_ptr(X.device))
        return out
    Xd = X.to(torch.float64)
    return Xd * (1.0 / torch.linalg.vector_norm(Xd, ord=p, dim=1))[:, None]


def axpby(alpha, X: Optional[torch.Tensor], beta, Y: torch.Tensor) -> torch.Tensor:
    """In place: Y = alpha·X + beta·Y, alpha / beta scalars or per-row [n] tensors
    (``BLAS.axpy``: beta = 1; ``BLAS.scal``: X = None)."""
    n, d = Y.shape
    if Y.is_cuda and Y.stride(1) == 1 and Y.dtype in (torch.float32, torch.float64, torch.bfloat16) and n:
        acc = _acc(Y.dtype)
        Xc = None
        if X is not None:
            Xc = X.to(Y.dtype)
            Xc = Xc if Xc.stride(1) == 1 else Xc.contiguous()
        ar = alpha.to(device=Y.device, dtype=acc).contiguous() if torch.is_tensor(alpha) else None
        br = beta.to(device=Y.device, dtype=acc).contiguous() if torch.is_tensor(beta) else None
        native.call("fmlx_blas_axpby", native.dtype_code(Y.dtype), native.ptr(Xc), Xc.stride(0) if Xc is not None else 0,
                    native.ptr(Y), Y.stride(0), n, d, 0.0 if ar is not None else float(alpha), native.ptr(ar),
                    0.0 if br is not None else float(beta), native.ptr(br), native.stream_ptr(Y.device))
        return Y
    a = alpha[:, None] if torch.is_tensor(alpha) else alpha
    b = beta[:, None] if torch.is_tensor(beta) else beta
    res = (a * X.to(torch.float64) if X is not None else 0) + b * Y.to(torch.float64)
    Y.copy_(res)
    return Y


def scal(alpha, Y: torch.Tensor) -> torch.Tensor:
    return axpby(0.0, None, alpha, Y)


def axpy(alpha, X: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
    return axpby(alpha, X, 1.0, Y)


def hdot(v, X):
    """Every row ∘ v (``BLAS.hDot`` with a broadcast vector; ElementwiseProduct)."""
    v = torch.as_tensor(v)
    if isinstance(X, SparseColumn):
        return csr_scale(X, col_scale=v)
    X = _rowmajor(X)
    n, d = X.shape
    if v.numel() != d:
        raise ValueError("Vector size mismatched.")
    if _dense_ok(X) and n:
        vd = v.to(device=X.device, dtype=torch.float64).contiguous()
        out = torch.empty((n, d), dtype=_acc(X.dtype), device=X.device)
        native.call("fmlx_blas_hdot", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), native.ptr(vd), n, d,
                    native.ptr(out), out.stride(0), native.stream_ptr(X.device))
        return out
    return X.to(torch.float64) * v.to(device=X.device, dtype=torch.float64)[None, :]


def csr_scale(X: SparseColumn, row_scale=None, col_scale=None) -> SparseColumn:
    """values · row_scale[row] · col_scale[index] (new column, same structure)."""
    if X.values.is_cuda and len(X):
        ip, ix, v = _csr_dev(X)
        out = torch.empty_like(v)
        rs = row_scale.to(device=v.device, dtype=torch.float64).contiguous() if row_scale is not None else None
        cs = torch.as_tensor(col_scale).to(device=v.device, dtype=torch.float64).contiguous() \
            if col_scale is not None else None
        native.call("fmlx_blas_csr_scale", native.dtype_code(v.dtype), native.ptr(ip), native.ptr(ix), native.ptr(v),
                    native.ptr(rs), native.ptr(cs), len(X), native.ptr(out), native.stream_ptr(v.device))
        return SparseColumn(X.indptr, X.indices, out, X.size)
    v = X.values.to(torch.float64)
    if row_scale is not None:
        rows = torch.repeat_interleave(torch.arange(len(X), device=v.device), X.indptr[1:] - X.indptr[:-1])
        v = v * row_scale.to(device=v.device, dtype=torch.float64)[rows]
    if col_scale is not None:
        v = v * torch.as_tensor(col_scale).to(device=v.device, dtype=torch.float64)[X.indices.long()]
    return SparseColumn(X.indptr, X.indices, v, X.size)


def csr_axpy_dense(alpha: float, X: SparseColumn, Y: torch.Tensor, k: Optional[int] = None) -> torch.Tensor:
    """Y[r, :k] += alpha · X[r, :k] for every row (``BLAS.axpy(a, sparse, dense, k)``); Y fp64."""
    k = X.size if k is None else int(k)
    if Y.dtype != torch.float64:
        raise TypeError("csr_axpy_dense accumulates into fp64 rows")
    if Y.is_cuda and len(X):
        ip, ix, v = _csr_dev(X)
        native.call("fmlx_blas_csr_axpy_dense", native.dtype_code(v.dtype), native.ptr(ip), native.ptr(ix),
                    native.ptr(v), float(alpha), len(X), k, native.ptr(Y), Y.stride(0), native.stream_ptr(Y.device))
        return Y
    rows = torch.repeat_interleave(torch.arange(len(X)), X.indptr[1:] - X.indptr[:-1])
    keep = X.indices.long() < k
    Y.index_put_((rows[keep], X.indices.long()[keep]), alpha * X.values.to(torch.float64)[keep], accumulate=True)
    return Y


def gather_cols(X: torch.Tensor, cols: Sequence[int]) -> torch.Tensor:
    """out[:, j] = X[:, cols[j]] (VectorSlicer on dense rows)."""
    X = _rowmajor(X) if X.dtype in (torch.float32, torch.float64, torch.bfloat16) else X
    idx = torch.as_tensor(list(cols), dtype=torch.int32, device=X.device)
    n = X.shape[0]
    if X.is_cuda and X.stride(1) == 1 and X.element_size() in (2, 4, 8) and n and len(idx):
        out = torch.empty((n, len(idx)), dtype=X.dtype, device=X.device)
        native.call("fmlx_blas_gather_cols", X.element_size(), native.ptr(X), X.stride(0), native.ptr(idx), n, len(idx),
                    native.ptr(out), native.stream_ptr(X.device))
        return out
    return X[:, idx.long()]


def gather_prod(X: torch.Tensor, terms: torch.Tensor) -> torch.Tensor:
    """out[:, j] = Π_q X[:, terms[j, q]] with a term index ≥ D meaning the constant 1
    (PolynomialExpansion's monomials) — one launch, no [n, T, degree] gather temporary."""
    n, d = X.shape
    T, deg = terms.shape
    if X.is_cuda and X.dtype in (torch.float32, torch.float64) and n and T:
        X = _rowmajor(X)
        tt = terms.to(device=X.device, dtype=torch.int32).contiguous()
        out = torch.empty((n, T), dtype=X.dtype, device=X.device)
        native.call("fmlx_blas_gather_prod", native.dtype_code(X.dtype), native.ptr(X), X.stride(0), d, native.ptr(tt),
                    deg, n, T, native.ptr(out), native.stream_ptr(X.device))
        return out
    Xp = torch.cat([X, torch.ones((n, 1), dtype=X.dtype, device=X.device)], dim=1)
    return Xp[:, terms.to(X.device).long().clamp(max=d)].prod(dim=2)


def interaction(mats: Sequence[torch.Tensor]) -> torch.Tensor:
    """Row-wise outer product of k dense columns, first input slowest (Interaction)."""
    mats = [m.to(torch.float64) if m.dim() == 2 else m.to(torch.float64)[:, None] for m in mats]
    mats = [m if m.stride(1) == 1 else m.contiguous() for m in mats]
    n = mats[0].shape[0]
    width = 1
    for m in mats:
        width *= m.shape[1]
    if mats[0].is_cuda and 1 <= len(mats) <= 8 and n:
        out = torch.empty((n, width), dtype=torch.float64, device=mats[0].device)
        ptrs = (ctypes.c_void_p * len(mats))(*[m.data_ptr() for m in mats])
        lds = (ctypes.c_long * len(mats))(*[m.stride(0) for m in mats])
        dims = (ctypes.c_long * len(mats))(*[m.shape[1] for m in mats])
        native.call("fmlx_blas_interaction", len(mats), ctypes.cast(ptrs, c_void_p), ctypes.cast(lds, c_void_p),
                    ctypes.cast(dims, c_void_p), n, native.ptr(out), native.stream_ptr(out.device))
        return out
    out = mats[0]
    for m in mats[1:]:
        out = (out[:, :, None] * m[:, None, :]).reshape(n, -1)
    return out
