"""Host-side vector and matrix types.

Mirrors the reference's ``Vector``/``DenseVector``/``SparseVector``/``DenseMatrix``/
``VectorWithNorm`` (flink-ml-core/src/main/java/org/apache/flink/ml/linalg/*.java).
These are the *row-level* types used by the user API and by model data; bulk data in
the engine lives in columnar device tensors (``flink_ml_amd.table``) and never goes
through these objects on the hot path.

Storage is numpy float64 (the reference is fp64 everywhere), so host parity tests are
bit-comparable with the Java implementation.
"""
from __future__ import annotations

import math
from typing import Iterable, Sequence, Union

import numpy as np


class Vector:
    """Abstract vector (reference ``linalg/Vector.java:25-45``)."""

    def size(self) -> int:
        raise NotImplementedError

    def get(self, i: int) -> float:
        raise NotImplementedError

    def set(self, i: int, value: float) -> None:
        raise NotImplementedError

    def to_array(self) -> np.ndarray:
        raise NotImplementedError

    def to_dense(self) -> "DenseVector":
        raise NotImplementedError

    def to_sparse(self) -> "SparseVector":
        raise NotImplementedError

    def clone(self) -> "Vector":
        raise NotImplementedError

    def __len__(self) -> int:
        return self.size()

    def __getitem__(self, i: int) -> float:
        return self.get(i)

    def __setitem__(self, i: int, value: float) -> None:
        self.set(i, value)

    # camelCase aliases used by code written against the Java/Python reference API
    def toArray(self):  # noqa: N802
        return self.to_array()

    def toDense(self):  # noqa: N802
        return self.to_dense()

    def toSparse(self):  # noqa: N802
        return self.to_sparse()


class DenseVector(Vector):
    """Dense vector backed by a float64 array (reference ``linalg/DenseVector.java:28``)."""

    __slots__ = ("values",)

    def __init__(self, values: Union[int, Sequence[float], np.ndarray]):
        if isinstance(values, (int, np.integer)):
            self.values = np.zeros(int(values), dtype=np.float64)
        else:
            self.values = np.ascontiguousarray(np.asarray(values, dtype=np.float64).reshape(-1))

    def size(self) -> int:
        return int(self.values.shape[0])

    def get(self, i: int) -> float:
        return float(self.values[i])

    def set(self, i: int, value: float) -> None:
        self.values[i] = value

    def to_array(self) -> np.ndarray:
        return self.values

    def to_dense(self) -> "DenseVector":
        return self

    def to_sparse(self) -> "SparseVector":
        idx = np.nonzero(self.values)[0].astype(np.int32)
        return SparseVector(self.size(), idx, self.values[idx])

    def clone(self) -> "DenseVector":
        return DenseVector(self.values.copy())

    def __eq__(self, other) -> bool:
        return isinstance(other, DenseVector) and np.array_equal(self.values, other.values)

    def __hash__(self) -> int:
        return hash(self.values.tobytes())

    def __repr__(self) -> str:
        return "[" + ", ".join(_fmt(v) for v in self.values) + "]"

    __str__ = __repr__


class SparseVector(Vector):
    """Sparse vector with sorted unique indices (reference ``linalg/SparseVector.java:30``).

    Construction sorts indices and validates they are unique and within ``[0, n)``
    (``SparseVector.java:133-181``).
    """

    __slots__ = ("n", "indices", "values")

    def __init__(self, n: int, indices: Sequence[int], values: Sequence[float]):
        self.n = int(n)
        idx = np.asarray(indices, dtype=np.int32).reshape(-1)
        val = np.asarray(values, dtype=np.float64).reshape(-1)
        if idx.shape[0] != val.shape[0]:
            raise ValueError("Indices size and values size should be the same.")
        if idx.shape[0] > 1 and np.any(idx[1:] <= idx[:-1]):
            order = np.argsort(idx, kind="stable")
            idx = idx[order]
            val = val[order]
        if idx.shape[0] > 0:
            if idx[0] < 0 or idx[-1] >= self.n:
                raise ValueError("Index out of bound.")
            if idx.shape[0] > 1 and np.any(idx[1:] == idx[:-1]):
                raise ValueError("Indices duplicated.")
        self.indices = np.ascontiguousarray(idx)
        self.values = np.ascontiguousarray(val)

    def size(self) -> int:
        return self.n

    def get(self, i: int) -> float:
        pos = np.searchsorted(self.indices, i)
        if pos < self.indices.shape[0] and self.indices[pos] == i:
            return float(self.values[pos])
        return 0.0

    def set(self, i: int, value: float) -> None:
        if i < 0 or i >= self.n:
            raise IndexError("Index out of bound.")
        pos = int(np.searchsorted(self.indices, i))
        if pos < self.indices.shape[0] and self.indices[pos] == i:
            self.values[pos] = value
        else:
            self.indices = np.insert(self.indices, pos, i).astype(np.int32)
            self.values = np.insert(self.values, pos, value)

    def to_array(self) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.float64)
        out[self.indices] = self.values
        return out

    def to_dense(self) -> DenseVector:
        return DenseVector(self.to_array())

    def to_sparse(self) -> "SparseVector":
        return self

    def clone(self) -> "SparseVector":
        return SparseVector(self.n, self.indices.copy(), self.values.copy())

    def __eq__(self, other) -> bool:
        return (
            isinstance(other, SparseVector)
            and self.n == other.n
            and np.array_equal(self.indices, other.indices)
            and np.array_equal(self.values, other.values)
        )

    def __hash__(self) -> int:
        return hash((self.n, self.indices.tobytes(), self.values.tobytes()))

    def __repr__(self) -> str:
        return "(%d, [%s], [%s])" % (
            self.n,
            ", ".join(str(int(i)) for i in self.indices),
            ", ".join(_fmt(v) for v in self.values),
        )

    __str__ = __repr__


class DenseMatrix:
    """Column-major dense matrix (reference ``linalg/DenseMatrix.java:30-90``)."""

    __slots__ = ("num_rows", "num_cols", "values")

    def __init__(self, num_rows: int, num_cols: int, values: Union[None, Sequence[float], np.ndarray] = None):
        self.num_rows = int(num_rows)
        self.num_cols = int(num_cols)
        if values is None:
            self.values = np.zeros(self.num_rows * self.num_cols, dtype=np.float64)
        else:
            v = np.asarray(values, dtype=np.float64).reshape(-1)
            if v.shape[0] != self.num_rows * self.num_cols:
                raise ValueError("Values array length mismatch.")
            self.values = np.ascontiguousarray(v)

    @staticmethod
    def from_rows_array(arr: np.ndarray) -> "DenseMatrix":
        arr = np.asarray(arr, dtype=np.float64)
        return DenseMatrix(arr.shape[0], arr.shape[1], arr.T.reshape(-1))

    def num_rows_(self) -> int:
        return self.num_rows

    def get(self, i: int, j: int) -> float:
        return float(self.values[self.num_rows * j + i])

    def to_numpy(self) -> np.ndarray:
        """Row-major [rows, cols] view."""
        return self.values.reshape(self.num_cols, self.num_rows).T

    def __eq__(self, other) -> bool:
        return (
            isinstance(other, DenseMatrix)
            and self.num_rows == other.num_rows
            and self.num_cols == other.num_cols
            and np.array_equal(self.values, other.values)
        )

    def __repr__(self) -> str:
        return "DenseMatrix(%d x %d)" % (self.num_rows, self.num_cols)


class VectorWithNorm:
    """A vector with its cached L2 norm (reference ``linalg/VectorWithNorm.java:27-39``)."""

    __slots__ = ("vector", "l2_norm")

    def __init__(self, vector: Vector, l2_norm: float = None):
        self.vector = vector
        if l2_norm is None:
            vals = vector.values
            l2_norm = math.sqrt(float(np.dot(vals, vals)))
        self.l2_norm = float(l2_norm)

    def __eq__(self, other) -> bool:
        return isinstance(other, VectorWithNorm) and self.vector == other.vector and self.l2_norm == other.l2_norm


class Vectors:
    """Factory helpers (reference ``linalg/Vectors.java:25-32``; Python API also accepts a
    dict or a list of (index, value) pairs for sparse vectors)."""

    @staticmethod
    def dense(*values) -> DenseVector:
        if len(values) == 1 and not isinstance(values[0], (int, float, np.floating, np.integer)):
            return DenseVector(values[0])
        return DenseVector(np.asarray(values, dtype=np.float64))

    @staticmethod
    def sparse(n: int, *args) -> SparseVector:
        if len(args) == 1:
            a = args[0]
            if isinstance(a, dict):
                items = sorted(a.items())
            else:
                items = sorted(list(a))
            idx = [int(k) for k, _ in items]
            val = [float(v) for _, v in items]
            return SparseVector(n, idx, val)
        if len(args) == 2:
            return SparseVector(n, args[0], args[1])
        raise TypeError("Vectors.sparse(n, indices, values) or Vectors.sparse(n, dict|pairs)")


def _fmt(v: float) -> str:
    v = float(v)
    if v == int(v) and abs(v) < 1e16:
        return "%.1f" % v
    return repr(v)


def as_vector(obj) -> Vector:
    """Coerces numbers/lists/arrays into a Vector (used for input-type conversion tests,
    reference ``LIBT/util/TestUtils.java:74``)."""
    if isinstance(obj, Vector):
        return obj
    if isinstance(obj, (list, tuple, np.ndarray)):
        return DenseVector(obj)
    raise TypeError("Cannot convert %r to Vector" % type(obj))


def stack_dense(vectors: Iterable[Vector], dim: int = None) -> np.ndarray:
    """Stacks vectors (dense or sparse) into a row-major float64 [n, dim] array."""
    vectors = list(vectors)
    if dim is None:
        dim = vectors[0].size() if vectors else 0
    out = np.zeros((len(vectors), dim), dtype=np.float64)
    for i, v in enumerate(vectors):
        if isinstance(v, DenseVector):
            out[i, :] = v.values
        else:
            out[i, v.indices] = v.values
    return out
