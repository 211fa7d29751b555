"""MinHash signatures (``csrc/minhash.hip``) with an exact int64 numpy path on CPU.

``minhash(X, a, b)`` returns fp64 [n, K] with K = numHashTables * numHashFunctionsPerTable, the
reference ``MinHashLSHModelData.hashFunction`` values flattened table-major.
"""
from __future__ import annotations

import numpy as np
import torch

from ..table import SparseColumn
from . import native
from .native import c_int, c_long, c_void_p

HASH_PRIME = 2038074743

native.register_kernel_sigs({
    "fmlx_minhash_csr": [c_void_p, c_void_p, c_long, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
})


def to_csr_sets(X) -> SparseColumn:
    """Nonzero pattern of a dense tensor or SparseColumn (``Vector.toSparse().indices``)."""
    if isinstance(X, SparseColumn):
        nz = X.values != 0
        if bool(nz.all()):
            return X
        rows = torch.repeat_interleave(torch.arange(len(X), device=X.values.device),
                                       (X.indptr[1:] - X.indptr[:-1]).to(X.values.device))[nz]
        indptr = torch.zeros(len(X) + 1, dtype=torch.int64, device=X.values.device)
        indptr[1:] = torch.cumsum(torch.bincount(rows, minlength=len(X)), 0)
        return SparseColumn(indptr, X.indices[nz], X.values[nz], X.size)
    nzr, nzc = torch.nonzero(X, as_tuple=True)
    indptr = torch.zeros(X.shape[0] + 1, dtype=torch.int64, device=X.device)
    indptr[1:] = torch.cumsum(torch.bincount(nzr, minlength=X.shape[0]), 0)
    return SparseColumn(indptr, nzc.to(torch.int32), X[nzr, nzc].to(torch.float64), X.shape[1])


def minhash(X, coef_a, coef_b) -> torch.Tensor:
    sets = to_csr_sets(X)
    n = len(sets)
    indptr = sets.indptr.to(torch.int64)
    if n and bool(((indptr[1:] - indptr[:-1]) == 0).any()):
        raise ValueError("Must have at least 1 non zero entry.")
    dev = sets.values.device
    K = len(coef_a)
    if dev.type == "cuda":
        a = torch.as_tensor(np.asarray(coef_a, dtype=np.int32), device=dev)
        b = torch.as_tensor(np.asarray(coef_b, dtype=np.int32), device=dev)
        ind = sets.indices.to(device=dev, dtype=torch.int32).contiguous()
        ip = indptr.to(dev).contiguous()
        out = torch.empty((n, K), dtype=torch.float64, device=dev)
        native.call("fmlx_minhash_csr", native.ptr(ip), native.ptr(ind) if ind.numel() else None, n, K,
                    native.ptr(a), native.ptr(b), native.ptr(out), native.stream_ptr(dev))
        return out
    ind = sets.indices.cpu().numpy().astype(np.int64)
    ip = indptr.cpu().numpy()
    a = np.asarray(coef_a, dtype=np.int64)
    b = np.asarray(coef_b, dtype=np.int64)
    if n == 0:
        return torch.zeros((0, K), dtype=torch.float64)
    h = ((1 + ind)[:, None] * a[None, :] + b[None, :]) % HASH_PRIME
    out = np.minimum.reduceat(h, ip[:-1], axis=0)
    return torch.from_numpy(out.astype(np.float64))


def jaccard_distance(x_idx: np.ndarray, y_idx: np.ndarray) -> float:
    """``MinHashLSHModelData.keyDistance``: 1 - |x ∩ y| / |x ∪ y| over nonzero index sets."""
    if len(x_idx) + len(y_idx) == 0:
        raise ValueError("The union of two input sets must have at least 1 elements")
    inter = len(np.intersect1d(x_idx, y_idx, assume_unique=True))
    return 1.0 - inter / (len(x_idx) + len(y_idx) - inter)
