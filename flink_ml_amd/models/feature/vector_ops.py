"""Stateless vector transformers (reference ``LIB/feature/{binarizer,bucketizer,dct,
elementwiseproduct,normalizer,polynomialexpansion,interaction,vectorassembler,vectorslicer}``).

All of them are batched tensor programs over the column (K16/K17 in SURVEY §2.1): they run on the
device-resident column in one or a few kernels instead of a per-row map function. Sparse inputs
stay sparse where the reference keeps them sparse.
"""
from __future__ import annotations

import functools
import math
from typing import List

import numpy as np
import torch

from ...ops import blas, native

from ...api.stage import Transformer
from ...common.param import HasHandleInvalid, HasInputCol, HasInputCols, HasOutputCol, HasOutputCols
from ...io import read_write as rw
from ...linalg.vectors import DenseVector, SparseVector, Vector
from ...ops import features as fo
from ...param.param import (BooleanParam, FloatArrayArrayParam, FloatArrayParam, FloatParam, IntArrayParam, IntParam,
                            ParamValidators, VectorParam)
from ...table import SparseColumn, Table
from .common import dense_input, row_ids, sparse_map_values, vector_input


# ------------------------------------------------------------------------------------ Binarizer
@rw.register_stage
class Binarizer(Transformer, HasInputCols, HasOutputCols):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.binarizer.Binarizer"
    THRESHOLDS = FloatArrayParam("thresholds", "The thresholds used to binarize continuous features.", None,
                                 ParamValidators.non_empty_array())

    def transform(self, *inputs):
        t = inputs[0]
        ins, outs, ths = self.get(self.INPUT_COLS), self.get(self.OUTPUT_COLS), self.get(self.THRESHOLDS)
        if len(ins) != len(outs) or len(ins) != len(ths):
            raise ValueError("The number of input columns, output columns and thresholds must be equal.")
        res = {}
        for c, o, th in zip(ins, outs, ths):
            col = t.column(c)
            if isinstance(col, torch.Tensor):
                res[o] = (col.to(torch.float64) > th).to(torch.float64)
            elif isinstance(col, SparseColumn):
                keep = col.values.to(torch.float64) > th
                rows = row_ids(col)[keep]
                counts = torch.bincount(rows, minlength=len(col))
                indptr = torch.cat([torch.zeros(1, dtype=torch.int64, device=counts.device), torch.cumsum(counts, 0)])
                res[o] = SparseColumn(indptr.to(col.indptr.device), col.indices[keep],
                                      torch.ones(int(keep.sum()), dtype=torch.float64, device=col.values.device),
                                      col.size)
            else:
                vals = []
                for v in col:
                    if isinstance(v, SparseVector):
                        m = v.values > th
                        vals.append(SparseVector(v.n, v.indices[m], np.ones(int(m.sum()))))
                    elif isinstance(v, Vector):
                        vals.append(DenseVector((v.values > th).astype(np.float64)))
                    else:
                        vals.append(1.0 if float(v) > th else 0.0)
                res[o] = vals
        return [t.with_columns(res)]


def _no_nan_device(x: torch.Tensor) -> bool:
    """No NaN in a device column: the valid count of the masked-sum kernel (csrc/colstats.hip)
    equals the length — one pass, no torch isnan / any kernels."""
    from .encoders import _valid_sum_count

    return int(_valid_sum_count(x.to(torch.float64), float("nan"))[1]) == x.shape[0]


# ------------------------------------------------------------------------------------ Bucketizer
native.register_kernel_sigs({"fmlx_bucketize": [native.c_void_p, native.c_long, native.c_void_p, native.c_int,
                                                 native.c_int, native.c_void_p, native.c_void_p, native.c_void_p,
                                                 native.c_void_p]})


def _bucketize_device(x: torch.Tensor, s: torch.Tensor, keep: bool, want_mask: bool):
    """(bucket index f64, invalid mask u8 or None when every value is valid) of a device column in
    one kernel pass (csrc/colstats.hip bucketize_kernel)."""
    x = x.contiguous()
    n, dev = x.shape[0], x.device
    out = torch.empty(n, dtype=torch.float64, device=dev)
    inv = torch.empty(n, dtype=torch.uint8, device=dev) if want_mask else None
    ninv = torch.zeros(1, dtype=torch.int32, device=dev)
    if n:
        native.call("fmlx_bucketize", native.ptr(x), n, native.ptr(s), len(s), int(keep), native.ptr(out),
                    native.ptr(inv) if inv is not None else None, native.ptr(ninv), native.stream_ptr(dev))
    return out, (inv if inv is not None else True) if int(ninv.item()) else None


@rw.register_stage
class Bucketizer(Transformer, HasInputCols, HasOutputCols, HasHandleInvalid):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.bucketizer.Bucketizer"
    SPLITS_ARRAY = FloatArrayArrayParam("splitsArray", "Array of split points for mapping continuous features into "
                                        "buckets.", None, ParamValidators.non_empty_array())

    def transform(self, *inputs):
        t = inputs[0]
        ins, outs, splits = self.get(self.INPUT_COLS), self.get(self.OUTPUT_COLS), self.get(self.SPLITS_ARRAY)
        hi = self.get(self.HANDLE_INVALID)
        keep_rows = None
        res = {}
        for c, o, sp in zip(ins, outs, splits):
            col = t.column(c)
            dev = col.device if isinstance(col, torch.Tensor) else torch.device("cpu")
            x = t.scalars(c, dtype=torch.float64, device=dev)
            s = torch.tensor(sp, dtype=torch.float64, device=dev)
            if dev.type == "cuda" and len(s):
                idx, invalid = _bucketize_device(x, s, hi == self.KEEP_INVALID, hi == self.SKIP_INVALID)
                if invalid is not None:  # (some invalid value)
                    if hi == self.ERROR_INVALID:
                        raise RuntimeError(
                            "The input contains invalid value. See handleInvalid parameter for more options.")
                    if hi == self.SKIP_INVALID:
                        inv_cpu = invalid.cpu().to(torch.bool)
                        keep_rows = ~inv_cpu if keep_rows is None else keep_rows & ~inv_cpu
                res[o] = idx
                continue
            pos = torch.searchsorted(s, x, right=False)  # first index with s[idx] >= x
            exact = (pos < len(s)) & (s[torch.clamp(pos, max=len(s) - 1)] == x)
            idx = torch.where(exact, torch.where(pos == len(s) - 1, pos - 1, pos), pos - 1).to(torch.float64)
            invalid = torch.isnan(x) | (~exact & ((pos == 0) | (pos == len(s))))
            if bool(invalid.any()):
                if hi == self.ERROR_INVALID:
                    raise RuntimeError("The input contains invalid value. See handleInvalid parameter for more options.")
                if hi == self.SKIP_INVALID:
                    inv_cpu = invalid.cpu()
                    keep_rows = ~inv_cpu if keep_rows is None else keep_rows & ~inv_cpu
                else:
                    idx = torch.where(invalid, torch.full_like(idx, float(len(s) - 1)), idx)
            res[o] = idx
        out = t.with_columns(res)
        if keep_rows is not None and not bool(keep_rows.all()):
            out = out.filter(keep_rows)
        return [out]


# ------------------------------------------------------------------------------------ DCT
def _dct_matrix(n: int) -> torch.Tensor:
    from ...ops.dct import dct_matrix

    return dct_matrix(n)  # orthonormal DCT-II basis (rows)


@rw.register_stage
class DCT(Transformer, HasInputCol, HasOutputCol):
    """Orthonormal DCT-II / DCT-III (JTransforms ``DoubleDCT_1D`` with scaled=true, DCT.java:103-123)
    as a product with the basis. K17 on the GPU: rows of n ≤ 128 go through the hand-written MFMA
    kernels with the basis resident in LDS (``ops/csrc/dct.hip``: f32, and f64 in parity mode on
    the f64 MFMA); wider rows and the CPU take the same product as a plain GEMM."""

    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.dct.DCT"
    INVERSE = BooleanParam("inverse", "Whether to perform the inverse DCT (true) or forward DCT (false).", False)

    def transform(self, *inputs):
        t = inputs[0]
        X = dense_input(t, self.get(self.INPUT_COL))
        n = X.shape[1]
        inv = self.get(self.INVERSE)
        dt = torch.float64 if X.dtype == torch.float64 or X.device.type == "cpu" else torch.float32
        Xd = X.to(dt)
        if Xd.is_cuda and 1 <= n <= 128:
            from ...ops.dct import dct_rows

            return [t.with_column(self.get(self.OUTPUT_COL), dct_rows(Xd, inv))]
        M = _dct_matrix(n).to(device=X.device, dtype=dt)
        out = Xd @ M if inv else Xd @ M.T
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


# ------------------------------------------------------------------------------------ ElementwiseProduct
@rw.register_stage
class ElementwiseProduct(Transformer, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.elementwiseproduct.ElementwiseProduct"
    SCALING_VEC = VectorParam("scalingVec", "The scaling vector to multiply with input vectors using hadamard product.",
                              None, ParamValidators.not_null())

    def transform(self, *inputs):
        t = inputs[0]
        X = vector_input(t, self.get(self.INPUT_COL))
        sv = self.get(self.SCALING_VEC)
        d = X.size if isinstance(X, SparseColumn) else X.shape[1]
        if sv.size() != d:
            raise ValueError("The scaling vector size is %d, which is not equal input vector size(%d)." % (sv.size(), d))
        # BLAS.hDot over the whole column (ops/blas.py: one HIP launch on the device)
        out = blas.hdot(torch.as_tensor(sv.to_array(), dtype=torch.float64), X)
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


# ------------------------------------------------------------------------------------ Normalizer
@rw.register_stage
class Normalizer(Transformer, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.normalizer.Normalizer"
    P = FloatParam("p", "The p norm value.", 2.0, ParamValidators.gt_eq(1.0))

    def transform(self, *inputs):
        t = inputs[0]
        X = vector_input(t, self.get(self.INPUT_COL))
        # BLAS.norm + BLAS.scal per row, fused (ops/blas.py normalize: one pass over each row)
        out = blas.normalize(X, self.get(self.P))
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


# ------------------------------------------------------------------------------------ PolynomialExpansion
def _poly_size(num: int, degree: int) -> int:
    if num == 0:
        return 1
    if num == 1 or degree == 1:
        return num + degree
    if degree > num:
        return _poly_size(degree, num)
    return math.comb(num + degree, degree)


@functools.lru_cache(maxsize=16)
def _poly_terms(d: int, degree: int) -> np.ndarray:
    """Monomial index lists in the reference's output order (PolynomialExpansion.java:217-245);
    padded with d (a column of ones)."""
    out = [None] * (_poly_size(d, degree) - 1)

    def expand(last, deg, mono, cur):
        if deg == 0 or last < 0:
            if cur >= 0:
                out[cur] = mono
        else:
            start = cur
            for i in range(deg + 1):
                start = expand(last - 1, deg - i, mono + [last] * i, start)
        return cur + _poly_size(last + 1, deg)

    expand(d - 1, degree, [], -1)
    arr = np.full((len(out), degree), d, dtype=np.int64)
    for j, m in enumerate(out):
        arr[j, : len(m)] = m
    return arr


@rw.register_stage
class PolynomialExpansion(Transformer, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.polynomialexpansion.PolynomialExpansion"
    DEGREE = IntParam("degree", "Degree of the polynomial expansion.", 2, ParamValidators.gt_eq(1))

    def transform(self, *inputs):
        t = inputs[0]
        col = t.column(self.get(self.INPUT_COL))
        sparse_in = isinstance(col, SparseColumn) or (isinstance(col, list) and col and isinstance(col[0], SparseVector))
        X = dense_input(t, self.get(self.INPUT_COL))
        Xd = X.to(torch.float64) if X.device.type == "cpu" else (X.float() if X.dtype == torch.bfloat16 else X)
        d = Xd.shape[1]
        terms = torch.as_tensor(_poly_terms(d, self.get(self.DEGREE)), device=Xd.device)
        out = blas.gather_prod(Xd, terms)  # one launch on the device (column index d = the constant 1)
        if sparse_in:
            out = SparseColumn.from_dense(out)
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


# ------------------------------------------------------------------------------------ Interaction
@rw.register_stage
class Interaction(Transformer, HasInputCols, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.interaction.Interaction"

    def transform(self, *inputs):
        t = inputs[0]
        mats = []
        sparse = False
        for c in self.get(self.INPUT_COLS):
            col = t.column(c)
            if isinstance(col, torch.Tensor) and col.dim() == 1:
                mats.append(col.to(torch.float64)[:, None])
            else:
                sparse = sparse or t.is_sparse(c)
                mats.append(dense_input(t, c).to(torch.float64))
        dev = mats[0].device
        out = blas.interaction([m.to(dev) for m in mats])  # one launch: row-wise outer products
        if sparse:
            out = SparseColumn.from_dense(out)
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


# ------------------------------------------------------------------------------------ VectorAssembler
@rw.register_stage
class VectorAssembler(Transformer, HasInputCols, HasOutputCol, HasHandleInvalid):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.vectorassembler.VectorAssembler"
    INPUT_SIZES = IntArrayParam("inputSizes", "Sizes of the input elements to be assembled.", None,
                                ParamValidators.non_empty_array())
    RATIO = 1.5

    def transform(self, *inputs):
        t = inputs[0]
        cols = self.get(self.INPUT_COLS)
        sizes = self.get(self.INPUT_SIZES)
        if len(sizes) != len(cols):
            raise ValueError("Input column names and input sizes should have the same length.")
        hi = self.get(self.HANDLE_INVALID)
        keep = hi == self.KEEP_INVALID
        # fast path: every input is a device dense/scalar column of the declared size
        fast = all(isinstance(t.column(c), torch.Tensor) for c in cols)
        if fast:
            parts, ok = [], torch.ones(t.num_rows, dtype=torch.bool, device=t.column(cols[0]).device)
            filtered = False
            for c, sz in zip(cols, sizes):
                col = t.column(c).to(torch.float64)
                col = col[:, None] if col.dim() == 1 else col
                if col.shape[1] != sz and not keep:
                    if hi == self.ERROR_INVALID:
                        raise RuntimeError("Vector assembler failed with exception : Input vector/number size does "
                                           "not meet with expected. Expected size: %d, actual size: %d."
                                           % (sz, col.shape[1]))
                    ok &= False  # skip: every row of a fixed-width column has the wrong size
                    filtered = True
                if col.shape[1] == 1 and not keep and not (col.is_cuda and _no_nan_device(col[:, 0])):
                    nan = torch.isnan(col[:, 0])
                    if bool(nan.any()):
                        filtered = True
                        if hi == self.ERROR_INVALID:
                            raise RuntimeError("Vector assembler failed with exception : Encountered NaN while "
                                               "assembling a row with handleInvalid = 'error'.")
                        ok &= ~nan
                parts.append(col)
            out = torch.cat(parts, dim=1)
            res = t.with_column(self.get(self.OUTPUT_COL), out)
            return [res if not filtered or bool(ok.all()) else res.filter(ok.cpu())]
        lists = [t.get_list(c) for c in cols]
        outs, keep_rows = [], []
        for r in range(t.num_rows):
            try:
                vals, size, nnz = [], 0, 0
                for i, (lst, sz) in enumerate(zip(lists, sizes)):
                    o = lst[r]
                    if o is None:
                        if not keep:
                            raise RuntimeError("Input column value is null.")
                        o = DenseVector(np.full(sz, np.nan)) if sz > 1 else float("nan")
                    if isinstance(o, Vector):
                        if o.size() != sz and not keep:
                            raise ValueError("Input vector/number size does not meet with expected.")
                        vals.append(o)
                        size += o.size()
                        nnz += o.indices.shape[0] if isinstance(o, SparseVector) else o.size()
                    else:
                        if sz != 1 and not keep:
                            raise ValueError("Input vector/number size does not meet with expected.")
                        if math.isnan(float(o)) and not keep:
                            raise RuntimeError("Encountered NaN while assembling a row with handleInvalid = 'error'.")
                        vals.append(float(o))
                        size += 1
                        nnz += 1
                dense = np.concatenate([v.to_array() if isinstance(v, Vector) else np.array([v]) for v in vals])
                outs.append(DenseVector(dense) if nnz * self.RATIO > size else DenseVector(dense).to_sparse())
                keep_rows.append(r)
            except Exception as e:  # noqa: BLE001 - mirrors the reference's catch-all
                if hi == self.ERROR_INVALID:
                    raise RuntimeError("Vector assembler failed with exception : %s" % e)
        res = t.take(keep_rows) if len(keep_rows) != t.num_rows else t
        return [res.with_column(self.get(self.OUTPUT_COL), outs)]


# ------------------------------------------------------------------------------------ VectorSlicer
@rw.register_stage
class VectorSlicer(Transformer, HasInputCol, HasOutputCol):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.vectorslicer.VectorSlicer"
    INDICES = IntArrayParam("indices", "An array of indices to select features from a vector column.", None)

    def transform(self, *inputs):
        t = inputs[0]
        idx = self.get(self.INDICES)
        if idx is None or len(idx) == 0:
            raise ValueError("Parameter indices's value should not be null")
        X = vector_input(t, self.get(self.INPUT_COL), exact=True)  # slicing moves values only
        d = X.size if isinstance(X, SparseColumn) else X.shape[1]
        if max(idx) >= d:
            raise ValueError("Index value %d is greater than vector size:%d" % (max(idx), d))
        if isinstance(X, SparseColumn):
            out = _slice_sparse(X, idx)
        else:
            out = blas.gather_cols(X, idx)
        return [t.with_column(self.get(self.OUTPUT_COL), out)]


def _slice_sparse(X: SparseColumn, idx) -> SparseColumn:
    """Selects columns of CSR rows without densifying (1M-wide rows stay sparse): old column →
    position in ``idx`` (or −1), kept non-zeros re-indexed and sorted within each row."""
    dev = X.values.device
    m = len(idx)
    pos = torch.full((X.size,), -1, dtype=torch.int64, device=dev)
    pos[torch.as_tensor(list(idx), dtype=torch.int64, device=dev)] = torch.arange(m, device=dev)
    counts = X.indptr[1:] - X.indptr[:-1]
    rows = torch.repeat_interleave(torch.arange(len(X), device=dev), counts.to(dev))
    newc = pos[X.indices.to(dev).long()]
    keep = newc >= 0
    rows, newc, vals = rows[keep], newc[keep], X.values.to(dev)[keep]
    order = torch.argsort(rows * m + newc)
    indptr = torch.zeros(len(X) + 1, dtype=torch.int64, device=dev)
    indptr[1:] = torch.cumsum(torch.bincount(rows, minlength=len(X)), 0)
    return SparseColumn(indptr, newc[order].to(torch.int32), vals[order], m)


def _indices_validator():
    from ...param.param import ParamValidator

    return ParamValidator(lambda v: v is not None and len(v) > 0 and len(set(v)) == len(v) and min(v) >= 0,
                          "distinct non-negative indices")


VectorSlicer.INDICES.validator = _indices_validator()
