"""Column functions (reference ``flink-ml-lib/.../Functions.java`` ``vectorToArray`` /
``arrayToVector`` and ``pyflink/ml/lib/functions.py``).

They work on a ``Table`` column (or directly on column data) and return the converted column:
dense vector columns stay device tensors (the conversion is a view/cast), sparse ones are
densified, list columns are converted element-wise.
"""
from __future__ import annotations

from typing import Union

import numpy as np
import torch

from .linalg.vectors import DenseVector, Vector
from .table import SparseColumn, Table


def _column(arg, col):
    return arg.column(col) if isinstance(arg, Table) else arg


def vector_to_array(data, col: str = None):
    """A column of ``Vector`` -> a column of double arrays (``Vector.toArray``)."""
    c = _column(data, col)
    if isinstance(c, torch.Tensor):
        return c.to(torch.float64)
    if isinstance(c, SparseColumn):
        return c.to_dense(torch.float64)
    return [None if v is None else (v.to_array() if isinstance(v, Vector) else np.asarray(v, dtype=np.float64))
            for v in c]


def array_to_vector(data, col: str = None):
    """A column of numeric arrays -> a column of ``DenseVector`` (as a dense device tensor when
    all rows have the same length)."""
    c = _column(data, col)
    if isinstance(c, torch.Tensor):
        return c.to(torch.float64) if c.dim() == 2 else c.to(torch.float64)[:, None]
    vecs = [None if a is None else DenseVector(np.asarray(a, dtype=np.float64)) for a in c]
    if vecs and all(v is not None for v in vecs) and len({v.size() for v in vecs}) == 1:
        return torch.from_numpy(np.stack([v.values for v in vecs]))
    return vecs


vectorToArray = vector_to_array
arrayToVector = array_to_vector
