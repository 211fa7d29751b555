"""Row-level BLAS on host vectors (reference ``linalg/BLAS.java:24-264``).

This is the *scalar* API used by model-data manipulation and by tests; the batched
device equivalents (K1/K2/K3 in SURVEY §2.1) live in ``flink_ml_amd.ops.blas`` and run as
HIP kernels on columnar tensors.
"""
from __future__ import annotations

import math

import numpy as np

from .vectors import DenseMatrix, DenseVector, SparseVector, Vector


def asum(x: DenseVector) -> float:
    return float(np.abs(x.values).sum())


def axpy(a: float, x: Vector, y: DenseVector, k: int = None) -> None:
    """y[:k] += a * x[:k]; sparse x stops at the first index >= k (``BLAS.java:206-220``)."""
    if k is None:
        if x.size() != y.size():
            raise ValueError("Vector size mismatched.")
        k = x.size()
    if x.size() < k or y.size() < k:
        raise ValueError("Illegal k for axpy.")
    if isinstance(x, SparseVector):
        cut = int(np.searchsorted(x.indices, k))
        np.add.at(y.values, x.indices[:cut], a * x.values[:cut])
    else:
        y.values[:k] += a * x.values[:k]


def dot(x: Vector, y: Vector) -> float:
    if x.size() != y.size():
        raise ValueError("Vector size mismatched.")
    if isinstance(x, SparseVector):
        if isinstance(y, SparseVector):
            _, ix, iy = np.intersect1d(x.indices, y.indices, assume_unique=True, return_indices=True)
            return float(np.dot(x.values[ix], y.values[iy]))
        return float(np.dot(x.values, y.values[x.indices]))
    if isinstance(y, SparseVector):
        return float(np.dot(y.values, x.values[y.indices]))
    return float(np.dot(x.values, y.values))


def hdot(x: Vector, y: Vector) -> None:
    """In-place Hadamard product ``y = x ∘ y`` (``BLAS.java:49-67,222-263``)."""
    if x.size() != y.size():
        raise ValueError("Vector size mismatched.")
    if isinstance(y, SparseVector):
        xv = x.to_array() if isinstance(x, SparseVector) else x.values
        y.values *= xv[y.indices]
    else:
        if isinstance(x, SparseVector):
            mask = np.zeros(y.size(), dtype=bool)
            mask[x.indices] = True
            y.values[x.indices] *= x.values
            y.values[~mask] = 0.0
        else:
            y.values *= x.values


def norm2(x: Vector) -> float:
    v = x.values
    return float(math.sqrt(float(np.dot(v, v))))


def norm(x: Vector, p: float) -> float:
    if p < 1.0:
        raise ValueError("p value must >= 1.0, but the current p is : %s" % p)
    data = np.abs(x.values)
    if p == 1.0:
        return float(data.sum())
    if p == 2.0:
        return norm2(x)
    if math.isinf(p):
        return float(data.max()) if data.size else 0.0
    return float(np.power(np.power(data, p).sum(), 1.0 / p))


def scal(a: float, x: Vector) -> None:
    x.values *= a


def gemv(alpha: float, matrix: DenseMatrix, trans: bool, x: DenseVector, beta: float, y: DenseVector) -> None:
    """y = alpha * op(M) x + beta * y with column-major M (``BLAS.java:179-204``)."""
    m = matrix.to_numpy()
    if trans:
        if not (matrix.num_rows == x.size() and matrix.num_cols == y.size()):
            raise ValueError("Matrix and vector size mismatched.")
        y.values[:] = alpha * (m.T @ x.values) + beta * y.values
    else:
        if not (matrix.num_rows == y.size() and matrix.num_cols == x.size()):
            raise ValueError("Matrix and vector size mismatched.")
        y.values[:] = alpha * (m @ x.values) + beta * y.values
