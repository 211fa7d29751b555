"""Helpers shared by the feature transformers."""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

from ... import config
from ...api.stage import Transformer
from ...common.param import HasInputCol, HasOutputCol
from ...io import serialization as ser
from ...linalg.vectors import DenseVector, SparseVector, Vector
from ...parallel import comm
from ...table import SparseColumn, Table


def dense_input(table: Table, col: str) -> torch.Tensor:
    """The vector column as a dense [n, d] tensor on the compute device (fp64 on CPU)."""
    return config.features_for_compute(table, col, allow_sparse=False)


def vector_input(table: Table, col: str, exact: bool = False):
    """Dense tensor or SparseColumn (kept sparse) on the compute device; ``exact`` keeps float64
    values unrounded (stages that only move values)."""
    return config.features_for_compute(table, col, allow_sparse=True, exact=exact)


def sparse_map_values(sc: SparseColumn, fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor]) -> SparseColumn:
    """Applies fn(values, indices) to a SparseColumn's values (structure unchanged)."""
    return SparseColumn(sc.indptr, sc.indices, fn(sc.values.to(torch.float64), sc.indices.long()), sc.size)


def row_ids(sc: SparseColumn) -> torch.Tensor:
    counts = (sc.indptr[1:] - sc.indptr[:-1]).to(sc.values.device)
    return torch.repeat_interleave(torch.arange(len(sc), device=sc.values.device), counts)


def all_reduce_stats(stats: dict) -> dict:
    """Combines per-rank column statistics (sum/sumsq/count add, min/max reduce)."""
    if not get_world_distributed():
        return stats
    out = dict(stats)
    for k in ("sum", "sumsq"):
        out[k] = comm.all_reduce_sum(stats[k].clone())
    out["min"] = comm.all_reduce(stats["min"].clone(), "min")
    out["max"] = comm.all_reduce(stats["max"].clone(), "max")
    out["count"] = int(comm.all_reduce_scalar(float(stats["count"]), "sum"))
    return out


def get_world_distributed() -> bool:
    from ...parallel.context import get_context

    return get_context().is_distributed


def vec_table_rows(vectors: Sequence[Vector], name: str) -> Table:
    return Table.from_rows([(v,) for v in vectors], [name])


def dense_vec(arr) -> DenseVector:
    if isinstance(arr, torch.Tensor):
        arr = arr.detach().to("cpu", torch.float64).numpy()
    return DenseVector(np.asarray(arr, dtype=np.float64))


def enc_dense(out, v):
    ser.write_dense_vector(out, v.to_dense() if isinstance(v, Vector) else DenseVector(v))


def dec_dense(inp):
    return ser.read_dense_vector(inp)


def out_dtype_tensor(x: torch.Tensor) -> torch.Tensor:
    return x


class VectorTransformerBase(Transformer, HasInputCol, HasOutputCol):
    """Row-aligned single-input/single-output vector transformer."""

    def _apply(self, X):
        raise NotImplementedError

    def transform(self, *inputs: Table):
        t = inputs[0]
        X = vector_input(t, self.get(self.INPUT_COL))
        return [t.with_column(self.get(self.OUTPUT_COL), self._apply(X))]


def select_by_indices(X, sorted_idx: Sequence[int]):
    """``VectorUtils.selectByIndices``: dense columns are gathered; a SparseColumn stays sparse
    (entries at unselected positions dropped, kept ones renumbered)."""
    if isinstance(X, SparseColumn):
        dev = X.values.device
        remap = torch.full((X.size,), -1, dtype=torch.int64, device=dev)
        if len(sorted_idx):
            remap[torch.as_tensor(sorted_idx, dtype=torch.int64, device=dev)] = torch.arange(len(sorted_idx),
                                                                                          device=dev)
        new = remap[X.indices.long()]
        keep = new >= 0
        rows = row_ids(X)[keep]
        indptr = torch.zeros(len(X) + 1, dtype=torch.int64, device=dev)
        indptr[1:] = torch.cumsum(torch.bincount(rows, minlength=len(X)), 0)
        return SparseColumn(indptr, new[keep].to(torch.int32), X.values[keep].to(torch.float64), len(sorted_idx))
    return X[:, torch.as_tensor(list(sorted_idx), dtype=torch.long, device=X.device)].to(torch.float64)
