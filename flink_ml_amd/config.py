"""Runtime configuration: device and numeric policy.

* ``FMLX_DEVICE`` — ``cpu`` forces the host path; default is ``cuda:<local_rank>`` when a GPU
  is visible.
* ``FMLX_COMPUTE_DTYPE`` — storage dtype for feature matrices handed to the kernels:
  ``fp64`` (parity mode: bit-level agreement with the reference's fp64 math; default on CPU),
  ``fp32`` (default on GPU) or ``bf16`` (fast path: halves HBM traffic; accumulation stays fp32).
  Tensors that are already device-resident in one of these dtypes are used as-is (no copy).
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch

from .parallel.context import get_context
from .table import SparseColumn, Table

_DTYPES = {"fp64": torch.float64, "fp32": torch.float32, "bf16": torch.bfloat16}
_OVERRIDE: Optional[str] = None


def compute_device() -> torch.device:
    return get_context().device


def compute_dtype_name() -> str:
    if _OVERRIDE is not None:
        return _OVERRIDE
    env = os.environ.get("FMLX_COMPUTE_DTYPE")
    if env:
        return env.lower()
    return "fp32" if compute_device().type == "cuda" else "fp64"


def compute_dtype() -> torch.dtype:
    return _DTYPES[compute_dtype_name()]


def acc_dtype() -> torch.dtype:
    return torch.float64 if compute_dtype() == torch.float64 else torch.float32


@contextlib.contextmanager
def dtype_policy(name: str):
    global _OVERRIDE
    old = _OVERRIDE
    _OVERRIDE = name
    try:
        yield
    finally:
        _OVERRIDE = old


def features_for_compute(table: Table, col: str, allow_sparse: bool = True, exact: bool = False):
    """The feature column as a device-resident dense tensor [n, d] or a ``SparseColumn``.
    ``exact``: for stages that only move values (slicing, assembling), float64 inputs keep float64
    on the device instead of taking the compute dtype, so no value changes."""
    dev = compute_device()
    c = table.column(col)
    if isinstance(c, torch.Tensor) and c.dim() == 2:
        if c.device == dev and c.dtype in (torch.float32, torch.float64, torch.bfloat16) and (
                dev.type == "cuda" or c.dtype == torch.float64):
            return c
        if exact and c.dtype in (torch.float32, torch.float64, torch.bfloat16):
            return c.to(device=dev)
        return c.to(device=dev, dtype=compute_dtype() if dev.type == "cuda" else torch.float64)
    wide = torch.float64 if exact or dev.type != "cuda" else None
    if allow_sparse and isinstance(c, SparseColumn):
        return c.to(device=dev, dtype=wide or acc_dtype())
    if allow_sparse and table.is_sparse(col):
        vecs = table.get_list(col)
        sc = SparseColumn.from_vectors([v.to_sparse() for v in vecs], table.vector_size(col))
        return sc.to(device=dev, dtype=wide or acc_dtype())
    return table.vectors_as_matrix(col, dtype=wide or compute_dtype(), device=dev)


def host_features_if_oversized(table: Table, col: str, allow_sparse: bool = False):
    """A host-resident feature column too large for the device — dense bytes in the compute dtype
    (or, with ``allow_sparse``, CSR bytes: indptr + indices + accumulation-dtype values) above the
    HBM budget (``FMLX_HBM_BUDGET``, else the device's free memory minus a margin) — converted but
    LEFT in host memory, when the compute device is a GPU: the bounded trainers then keep what
    fits resident and stream the rest (common/outofcore.py). None otherwise (the column goes to
    the device as usual)."""
    from .common.outofcore import hbm_budget

    dev = compute_device()
    c = table.column(col)
    if dev.type != "cuda":
        return None
    if allow_sparse and isinstance(c, SparseColumn) and not c.values.is_cuda:
        acc = acc_dtype()
        need = c.indptr.numel() * 8 + c.indices.numel() * (4 + torch.empty(0, dtype=acc).element_size())
        budget = hbm_budget(dev)
        if budget is None or need <= budget:
            return None
        return c.to(dtype=acc)
    if not isinstance(c, torch.Tensor) or c.dim() != 2 or c.is_cuda:
        return None
    dt = compute_dtype()
    budget = hbm_budget(dev)
    if budget is None or c.shape[0] * c.shape[1] * torch.empty(0, dtype=dt).element_size() <= budget:
        return None
    return c.to(dt).contiguous() if c.dtype != dt or not c.is_contiguous() else c
