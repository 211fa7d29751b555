"""Categorical / discretising encoders (reference ``LIB/feature/{onehotencoder,stringindexer,
vectorindexer,kbinsdiscretizer,imputer}``).

Numeric work stays on the rank's device and only fixed-size statistics cross ranks:

* OneHotEncoder: per-column max index is a device ``max`` + all-reduce; the transform builds the
  one-hot SparseColumn (indptr = cumsum(valid)) with no per-row host loop.
* StringIndexer on numeric columns maps unique values (device ``unique``) to strings once and
  then indexes rows with a device ``searchsorted`` lookup table; string columns use a host dict.
* VectorIndexer counts distinct values per column with a single column-wise device sort.
* KBinsDiscretizer bins every column with one batched ``searchsorted`` over padded edges.
* Imputer computes mean / median / most-frequent surrogates from device-side reductions.

Model-data records use the reference encoders so saved models are interchangeable:
OneHotEncoder (Kryo ``writeInt`` pairs), StringIndexer (``IntSerializer`` + ``StringArraySerializer``),
VectorIndexer (``MapSerializer<Integer, Map<Double, Integer>>``), KBinsDiscretizer (``double[][]``),
Imputer (``MapSerializer<String, Double>``); map entries are written in Java ``HashMap`` order.
"""
from __future__ import annotations

import math
from collections import Counter
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ... import config
from ...api.stage import Estimator
from ...common.param import HasHandleInvalid, HasInputCol, HasInputCols, HasOutputCol, HasOutputCols, HasRelativeError
from ...io import read_write as rw
from ...io import serialization as ser
from ...linalg.vectors import DenseVector, SparseVector, Vector
from ...ops import features as fo
from ...ops import native
from ...param.param import BooleanParam, FloatParam, IntParam, ParamValidators, StringParam
from ...parallel import comm
from ...parallel import datastream as ds
from ...table import SparseColumn, StringColumn, Table, first_occurrence
from ...utils.strtable import StrTable, hashmap_order_from_hashes
from ...utils.java import (java_double_hash, java_hashmap_order, java_int_hash, java_number_to_string,
                           java_string_hash)
from ..base import ModelWithData
from ..linear import rw_update
from .common import get_world_distributed
from .scalers import exact_quantiles


def _dev():
    return config.compute_device()


def _numeric_col(t: Table, col: str) -> torch.Tensor:
    c = t.column(col)
    if isinstance(c, StringColumn) and len(c) > 0:
        # numeric strings: parse each distinct value once, gather by code
        try:
            lut = torch.tensor([float(w) for w in c.vocab], dtype=torch.float64)
        except (TypeError, ValueError):
            raise RuntimeError("Column %s is not numeric." % col) from None
        return lut.to(c.codes.device)[c.codes.long()]
    if isinstance(c, torch.Tensor):
        if c.dim() != 1:
            raise ValueError("Column %s is not a scalar column" % col)
        return c
    vals = [float("nan") if v is None else float(v) for v in c]
    return torch.tensor(vals, dtype=torch.float64)


def _ordered_map(m: Dict, hash_fn) -> Dict:
    """Re-inserts ``m`` in Java ``HashMap`` iteration order (insertion order = current order)."""
    return {k: m[k] for k in java_hashmap_order(list(m.keys()), hash_fn)}


# ================================================================================ OneHotEncoder
class OneHotEncoderParams(HasInputCols, HasOutputCols, HasHandleInvalid):
    DROP_LAST = BooleanParam("dropLast", "Whether to drop the last category.", True)


@rw.register_stage
class OneHotEncoderModel(ModelWithData, OneHotEncoderParams):
    """``OneHotEncoderModel.java``: column i value v -> SparseVector(size_i, [v], [1.0]); with
    dropLast the last category (v == size_i) maps to the empty vector."""

    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.onehotencoder.OneHotEncoderModel"
    MODEL_DATA_COLUMNS = ("f0", "f1")

    @staticmethod
    def encode_record(out, row):
        out.write_int(int(row[0]))  # Kryo Output.writeInt is big-endian
        out.write_int(int(row[1]))

    @staticmethod
    def decode_record(inp):
        return (inp.read_int(), inp.read_int())

    def _build_state(self, rows):
        sizes = [0] * len(rows)
        off = 0 if self.get(self.DROP_LAST) else 1
        for ci, mx in rows:
            sizes[int(ci)] = int(mx) + off
        return sizes

    def transform(self, *inputs):
        if self.get(self.HANDLE_INVALID) != self.ERROR_INVALID:
            raise ValueError("OneHotEncoderModel only supports handleInvalid = 'error'.")
        t = inputs[0]
        ins, outs = self.get(self.INPUT_COLS), self.get(self.OUTPUT_COLS)
        if len(ins) != len(outs):
            raise ValueError("The number of input columns and output columns must be equal.")
        sizes = self._model_state()
        res = {}
        for i, (c, o) in enumerate(zip(ins, outs)):
            x = _numeric_col(t, c)
            xi = x.to(torch.int64)
            if bool((xi.to(x.dtype) != x).any()):
                bad = x[xi.to(x.dtype) != x][0].item()
                raise ValueError("Value %s cannot be parsed as indexed integer." % bad)
            size = sizes[i]
            if bool(((xi < 0) | (xi > size)).any()):
                raise IndexError("Index out of bounds for one-hot vector of size %d." % size)
            valid = xi < size
            indptr = torch.zeros(len(xi) + 1, dtype=torch.int64, device=xi.device)
            indptr[1:] = torch.cumsum(valid.to(torch.int64), 0)
            idx = xi[valid].to(torch.int32)
            res[o] = SparseColumn(indptr, idx, torch.ones(idx.numel(), dtype=torch.float64, device=xi.device), size)
        return [t.with_columns(res)]


@rw.register_stage
class OneHotEncoder(Estimator, OneHotEncoderParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.onehotencoder.OneHotEncoder"

    def fit(self, *inputs):
        if self.get(self.HANDLE_INVALID) != self.ERROR_INVALID:
            raise ValueError("OneHotEncoder only supports handleInvalid = 'error'.")
        t = inputs[0]
        cols = self.get(self.INPUT_COLS)
        maxes = []
        for c in cols:
            x = _numeric_col(t, c)
            if x.is_cuda and x.numel() and x.dtype in (torch.float32, torch.float64):
                # one library reduction (min, max, any non-integer / non-finite) answers the checks
                # for valid input; torch's compare / any kernels would load their code objects
                # lazily inside the first fit of a process
                from ...ops import catstats

                mn, mxv, non = catstats.flags(x)
                if not non and mn >= 0.0 and mxv < 2.0 ** 62:
                    maxes.append(int(mxv))
                    continue
            xi = x.to(torch.int64)
            if x.numel() and bool((xi.to(x.dtype) != x).any()):
                bad = x[xi.to(x.dtype) != x][0].item()
                raise ValueError("Value %s cannot be parsed as indexed integer." % bad)
            if x.numel() and bool((xi < 0).any()):
                raise ValueError("Negative value not supported.")
            maxes.append(int(xi.max().item()) if xi.numel() else -(1 << 31))
        mx = torch.tensor(maxes, dtype=torch.int64)
        if get_world_distributed():
            mx = comm.all_reduce(mx, "max")
        rows = [(i, int(v)) for i, v in enumerate(mx.tolist())]
        m = OneHotEncoderModel().set_model_data(OneHotEncoderModel.make_model_data_table(rows))
        rw_update(m, self)
        return m


# ================================================================================ StringIndexer
ARBITRARY_ORDER = "arbitrary"
FREQUENCY_DESC_ORDER = "frequencyDesc"
FREQUENCY_ASC_ORDER = "frequencyAsc"
ALPHABET_DESC_ORDER = "alphabetDesc"
ALPHABET_ASC_ORDER = "alphabetAsc"


class StringIndexerModelParams(HasInputCols, HasOutputCols, HasHandleInvalid):
    pass


class StringIndexerParams(StringIndexerModelParams):
    ARBITRARY_ORDER = ARBITRARY_ORDER
    FREQUENCY_DESC_ORDER = FREQUENCY_DESC_ORDER
    FREQUENCY_ASC_ORDER = FREQUENCY_ASC_ORDER
    ALPHABET_DESC_ORDER = ALPHABET_DESC_ORDER
    ALPHABET_ASC_ORDER = ALPHABET_ASC_ORDER
    STRING_ORDER_TYPE = StringParam("stringOrderType", "How to order strings of each column.", ARBITRARY_ORDER,
                                    ParamValidators.in_array(ARBITRARY_ORDER, FREQUENCY_DESC_ORDER,
                                                             FREQUENCY_ASC_ORDER, ALPHABET_DESC_ORDER,
                                                             ALPHABET_ASC_ORDER))


def _java_str_key(s: str) -> bytes:
    # String.compareTo compares UTF-16 code units
    return s.encode("utf-16-be")


def _string_counts_table(t: Table, col: str):
    """This rank's distinct strings of a column (numbers via String.valueOf) as a StrTable, their
    counts and first-seen row positions (the insertion order of the reference's per-partition
    ``Map<String, Long>``)."""
    c = t.column(col)
    if isinstance(c, StringColumn) and len(c) > 0:
        try:
            tab = StrTable.from_strings(c.vocab)
        except TypeError:
            raise RuntimeError("The input column only supports string and numeric type.") from None
        # counts and first occurrences per vocabulary entry by code on the device
        V = len(c.vocab)
        from ...ops import catstats

        got = catstats.code_counts_first(c.codes.to(config.compute_device()), V)
        if got is not None:  # one kernel pass; the [V] results ordered on the host
            cnt_h, first_h = got
            present = np.nonzero(cnt_h > 0)[0]
            present = present[np.argsort(first_h[present], kind="stable")]
            return tab.take(present), cnt_h[present], first_h[present]
        codes = c.codes.to(config.compute_device()).long()
        cnt = torch.bincount(codes, minlength=V)
        first = first_occurrence(codes, V)
        present = torch.nonzero(cnt > 0).reshape(-1)
        # present entries in first-seen order (the device sorts; first positions are distinct)
        present = present[torch.argsort(first[present])]
        return tab.take(present.cpu().numpy()), cnt[present].cpu().numpy(), first[present].cpu().numpy()
    if isinstance(c, torch.Tensor):
        if c.dim() != 1:
            raise RuntimeError("The input column only supports string and numeric type.")
        u, inv, cnt = torch.unique(c, return_inverse=True, return_counts=True)
        first = torch.full((u.numel(),), c.numel(), dtype=torch.int64, device=c.device)
        first.scatter_reduce_(0, inv, torch.arange(c.numel(), device=c.device), "amin")
        is_int = not c.dtype.is_floating_point
        strs = [str(int(v)) if is_int else java_number_to_string(v) for v in u.tolist()]
        return StrTable.from_strings(strs), cnt.cpu().numpy(), first.cpu().numpy()
    counts: Dict[str, int] = {}
    firsts: Dict[str, int] = {}
    for r, v in enumerate(c):
        if isinstance(v, str):
            w = v
        elif isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool):
            w = java_number_to_string(v.item() if hasattr(v, "item") else v)
        else:
            raise RuntimeError("The input column only supports string and numeric type.")
        if w not in counts:
            counts[w] = 0
            firsts[w] = r
        counts[w] += 1
    keys = list(counts)
    return (StrTable.from_strings(keys), np.array([counts[k] for k in keys], dtype=np.int64),
            np.array([firsts[k] for k in keys], dtype=np.int64))


def _string_counts(t: Table, col: str) -> Dict[str, int]:
    """Per-rank ``Map<String, Long>`` of a column in first-seen order (numbers via String.valueOf)."""
    tab, cnt, first = _string_counts_table(t, col)
    tab, sums, _ = _local_merge(tab, cnt, first)
    return dict(zip(tab.strings(), sums[:, 0].astype(np.int64).tolist()))


def _local_merge(tab: StrTable, cnt: np.ndarray, first: np.ndarray):
    order = np.argsort(first, kind="stable")
    tab, cnt, first = tab.take(order), cnt[order], first[order]
    rep = tab.first_of_equal()
    if len(tab) and not np.array_equal(rep, np.arange(len(tab))):
        uniq, inv = np.unique(rep, return_inverse=True)
        s2 = np.zeros((uniq.shape[0], 1), dtype=np.float64)
        np.add.at(s2[:, 0], inv, cnt)
        return tab.take(uniq), s2, first[uniq]
    return tab, cnt.astype(np.float64)[:, None], first


def order_string_table(tab: StrTable, counts: np.ndarray, order: str) -> np.ndarray:
    """Positions of ``tab``'s strings (inserted in table order into a Java HashMap) in the
    requested StringIndexer order (``StringIndexer.java:160-178``): HashMap iteration order,
    then a stable sort by frequency, or ``String.compareTo`` order."""
    if order == ALPHABET_ASC_ORDER:
        return tab.argsort(False)
    if order == ALPHABET_DESC_ORDER:
        return tab.argsort(True)
    hm = hashmap_order_from_hashes(tab.java_hashes())
    if order == FREQUENCY_ASC_ORDER:
        return hm[np.argsort(counts[hm], kind="stable")]
    if order == FREQUENCY_DESC_ORDER:
        return hm[np.argsort(-counts[hm], kind="stable")]
    if order != ARBITRARY_ORDER:
        raise ValueError("Unsupported stringOrderType type: %s." % order)
    return hm


def _order_strings(counts: Dict[str, int], order: str) -> List[str]:
    keys = list(counts)
    tab = StrTable.from_strings(keys)
    perm = order_string_table(tab, np.array([counts[k] for k in keys], dtype=np.int64), order)
    return [keys[i] for i in perm.tolist()]


class _LookupTable:
    """string → index of one model array, as the reference's ``HashMap`` built by putting the
    array's strings in order (a later duplicate overwrites an earlier one): a native hash join for
    batches of distinct strings, a dict only for the per-row list path."""

    def __init__(self, arr: Sequence[str]):
        self.arr = list(arr)
        self._rev = None
        self._dict = None

    def __len__(self) -> int:
        return len(self.arr)

    def lookup(self, queries: StrTable) -> np.ndarray:
        """Index of every query string (−1 if absent)."""
        if self._rev is None:
            self._rev = StrTable.from_strings(self.arr[::-1])
        r = self._rev.lookup(queries)
        return np.where(r >= 0, len(self.arr) - 1 - r, -1)

    @property
    def dict(self) -> Dict[str, float]:
        if self._dict is None:
            self._dict = {w: float(i) for i, w in enumerate(self.arr)}
        return self._dict


class _StringArraysModel(ModelWithData):
    MODEL_DATA_COLUMNS = ("stringArrays",)

    @staticmethod
    def encode_record(out, row):
        arrays = row[0]
        out.write_int(len(arrays))
        for a in arrays:
            ser.write_string_array(out, list(a))

    @staticmethod
    def decode_record(inp):
        return ([ser.read_string_array(inp) for _ in range(inp.read_int())],)

    @classmethod
    def make_model_data_table(cls, rows, strings_only: bool = False):
        """``strings_only``: the arrays already hold str objects only (no String.valueOf pass)."""
        def as_str(v):
            return v if isinstance(v, str) else java_number_to_string(v)

        if strings_only:
            return Table({"stringArrays": [[list(a) for a in r[0]] for r in rows]}, num_rows=len(rows))
        return Table({"stringArrays": [[[as_str(v) for v in a] for a in r[0]] for r in rows]}, num_rows=len(rows))


@rw.register_stage
class StringIndexerModel(_StringArraysModel, StringIndexerModelParams):
    """``StringIndexerModel.java``: string (or String.valueOf(number)) -> double index;
    unseen values follow handleInvalid (error / skip the row / keep -> numLabels)."""

    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.stringindexer.StringIndexerModel"

    def _build_state(self, rows):
        # one native string table per input column (first index of equal strings wins, like the
        # reference's HashMap built in array order); the per-row dict is made only if needed
        return [_LookupTable(arr) for arr in rows[0][0]]

    def transform(self, *inputs):
        t = inputs[0]
        ins, outs = self.get(self.INPUT_COLS), self.get(self.OUTPUT_COLS)
        hi = self.get(self.HANDLE_INVALID)
        maps = self._model_state()
        keep_rows = torch.ones(t.num_rows, dtype=torch.bool)
        res = {}
        for i, (c, o) in enumerate(zip(ins, outs)):
            m = maps[i]
            col = t.column(c)
            if isinstance(col, StringColumn):
                # look up each distinct string once (native hash join), gather by code
                codes = col.codes.to(config.compute_device()).long()
                keys = col.vocab
                try:
                    qtab = StrTable.from_strings(keys)
                except TypeError:
                    raise RuntimeError("The input column only supports string and numeric type.") from None
                lut = torch.from_numpy(m.lookup(qtab).astype(np.float64)).to(codes.device)
                idx = lut[codes]
                bad = idx < 0
                if bool(bad.any()):
                    if hi == self.ERROR_INVALID:
                        k = keys[int(codes[bad][0])]
                        raise RuntimeError("The input contains unseen string: %s. See handleInvalid parameter for "
                                           "more options." % k)
                    if hi == self.SKIP_INVALID:
                        keep_rows &= ~bad.cpu()
                    idx = torch.where(bad, torch.full_like(idx, float(len(m))), idx)
                res[o] = idx
            elif isinstance(col, torch.Tensor) and col.dim() == 1:
                u, inv = torch.unique(col, return_inverse=True)
                is_int = not col.dtype.is_floating_point
                keys = [str(int(v)) if is_int else java_number_to_string(v) for v in u.tolist()]
                lut = torch.from_numpy(m.lookup(StrTable.from_strings(keys)).astype(np.float64)).to(col.device)
                idx = lut[inv]
                bad = idx < 0
                if bool(bad.any()):
                    if hi == self.ERROR_INVALID:
                        k = keys[int(inv[bad][0])]
                        raise RuntimeError("The input contains unseen string: %s. See handleInvalid parameter for "
                                           "more options." % k)
                    if hi == self.SKIP_INVALID:
                        keep_rows &= ~bad.cpu()
                    idx = torch.where(bad, torch.full_like(idx, float(len(m))), idx)
                res[o] = idx
            else:
                vals = []
                for r, v in enumerate(col):
                    if isinstance(v, str):
                        s = v
                    elif isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool):
                        s = java_number_to_string(v.item() if hasattr(v, "item") else v)
                    else:
                        raise RuntimeError("The input column only supports string and numeric type.")
                    if s in m.dict:
                        vals.append(m.dict[s])
                    elif hi == self.ERROR_INVALID:
                        raise RuntimeError("The input contains unseen string: %s. See handleInvalid parameter for "
                                           "more options." % s)
                    elif hi == self.SKIP_INVALID:
                        keep_rows[r] = False
                        vals.append(-1.0)
                    else:
                        vals.append(float(len(m)))
                res[o] = torch.tensor(vals, dtype=torch.float64)
        out = t.with_columns(res)
        if not bool(keep_rows.all()):
            out = out.filter(keep_rows)
        return [out]


@rw.register_stage
class StringIndexer(Estimator, StringIndexerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.stringindexer.StringIndexer"

    def fit(self, *inputs):
        t = inputs[0]
        cols = self.get(self.INPUT_COLS)
        if len(cols) != len(self.get(self.OUTPUT_COLS)):
            raise ValueError("The number of input columns and output columns must be equal.")
        arrays = []
        dist = get_world_distributed()
        for c in cols:
            # per-rank (string, count, first position) tables merged by a keyed shuffle of the
            # strings (all-to-all to the owner of each string's hash, owners' maps all-gathered)
            err = None
            try:
                tab, cnt, first = _string_counts_table(t, c)
            except RuntimeError as e:  # a bad column on one rank: every rank raises, none blocks
                err = e
            if dist and comm.all_reduce_scalar(0.0 if err else 1.0, "min") < 1.0:
                raise err or RuntimeError("The input column only supports string and numeric type.")
            if err is not None:
                raise err
            tab, sums, _ = ds.reduce_strings_by_key(tab, cnt[:, None], first)
            perm = order_string_table(tab, sums[:, 0], self.get(self.STRING_ORDER_TYPE))
            arrays.append(tab.take_strings(perm))
        m = StringIndexerModel().set_model_data(StringIndexerModel.make_model_data_table([(arrays,)],
                                                                                         strings_only=True))
        rw_update(m, self)
        return m


@rw.register_stage
class IndexToStringModel(_StringArraysModel, HasInputCols, HasOutputCols):
    """``IndexToStringModel.java``: integer index -> string of the StringIndexerModel data."""

    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.stringindexer.IndexToStringModel"

    def transform(self, *inputs):
        t = inputs[0]
        arrays = self.model_data_rows()[0][0]
        res = {}
        for i, (c, o) in enumerate(zip(self.get(self.INPUT_COLS), self.get(self.OUTPUT_COLS))):
            # the output is dictionary-encoded: codes = the indices (validated on the device),
            # dictionary = the model array — no per-row strings are built
            ids = _numeric_col(t, c).to(torch.int64)
            arr = arrays[i]
            bad = (ids < 0) | (ids >= len(arr))
            if bool(bad.any()):
                raise RuntimeError("The input contains unseen index: %d." % int(ids[bad][0]))
            res[o] = StringColumn(ids.to(torch.int32), arr)
        return [t.with_columns(res)]


# ================================================================================ VectorIndexer
class VectorIndexerModelParams(HasInputCol, HasOutputCol, HasHandleInvalid):
    pass


class VectorIndexerParams(VectorIndexerModelParams):
    MAX_CATEGORIES = IntParam("maxCategories", "Threshold for the number of values a categorical feature can take "
                              "(>= 2). If a feature is found to have > maxCategories values, then it is declared "
                              "continuous.", 20, ParamValidators.gt_eq(2))


def _dense_matrix(t: Table, col: str) -> torch.Tensor:
    c = t.column(col)
    if isinstance(c, SparseColumn):
        return c.to_dense(torch.float64)
    return config.features_for_compute(t, col, allow_sparse=False)


def _category_map(values: Sequence[float]) -> Dict[float, int]:
    """``VectorIndexer.ModelGenerator``: sorted distinct values with 0.0 (if present) moved to index 0."""
    vals = sorted(values)
    if 0.0 in vals:
        vals.remove(0.0)
        vals = [0.0] + vals
    return {v: i for i, v in enumerate(vals)}


@rw.register_stage
class VectorIndexerModel(ModelWithData, VectorIndexerModelParams):
    """``VectorIndexerModel.java``: categorical columns' values -> category indices."""

    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.vectorindexer.VectorIndexerModel"
    MODEL_DATA_COLUMNS = ("categoryMaps",)

    @staticmethod
    def encode_record(out, row):
        maps = _ordered_map({int(k): v for k, v in row[0].items()}, java_int_hash)
        ser.write_map(out, maps, lambda o, k: o.write_int(k),
                      lambda o, m: ser.write_map(o, _ordered_map(m, java_double_hash), lambda o2, x: o2.write_double(x),
                                                 lambda o2, x: o2.write_int(int(x))))

    @staticmethod
    def decode_record(inp):
        return (ser.read_map(inp, lambda i: i.read_int(),
                             lambda i: ser.read_map(i, lambda i2: i2.read_double(), lambda i2: i2.read_int())),)

    @classmethod
    def make_model_data_table(cls, rows):
        return Table({"categoryMaps": [r[0] for r in rows]}, num_rows=len(rows))

    def _build_state(self, rows):
        maps = rows[0][0]
        state = []
        for ci in sorted(maps.keys()):
            m = maps[ci]
            keys = sorted(m.keys())
            state.append((int(ci), torch.tensor(keys, dtype=torch.float64),
                          torch.tensor([float(m[k]) for k in keys], dtype=torch.float64), len(m)))
        return state

    def transform(self, *inputs):
        t = inputs[0]
        col = t.column(self.get(self.INPUT_COL))
        was_sparse = isinstance(col, SparseColumn) or (isinstance(col, list) and col and isinstance(col[0],
                                                                                                     SparseVector))
        X = _dense_matrix(t, self.get(self.INPUT_COL)).to(torch.float64)
        out = X.clone()
        hi = self.get(self.HANDLE_INVALID)
        keep = torch.ones(X.shape[0], dtype=torch.bool, device=X.device)
        for ci, keys, vals, size in self._model_state():
            keys, vals = keys.to(X.device), vals.to(X.device)
            x = X[:, ci].contiguous()
            pos = torch.clamp(torch.searchsorted(keys, x), max=keys.numel() - 1)
            hit = keys[pos] == x
            if not bool(hit.all()):
                if hi == self.ERROR_INVALID:
                    raise RuntimeError("The input contains unseen double: %s. See handleInvalid parameter for more "
                                       "options." % java_number_to_string(float(x[~hit][0])))
                if hi == self.SKIP_INVALID:
                    keep &= hit
            out[:, ci] = torch.where(hit, vals[pos], torch.full_like(x, float(size)))
        if was_sparse:
            res_col = SparseColumn.from_dense(out)
        else:
            res_col = out
        res = t.with_column(self.get(self.OUTPUT_COL), res_col)
        if not bool(keep.all()):
            res = res.filter(keep.cpu())
        return [res]


@rw.register_stage
class VectorIndexer(Estimator, VectorIndexerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.vectorindexer.VectorIndexer"

    def fit(self, *inputs):
        t = inputs[0]
        max_cat = self.get(self.MAX_CATEGORIES)
        X = _dense_matrix(t, self.get(self.INPUT_COL)).to(torch.float64)
        n, d = X.shape
        dist = get_world_distributed()
        # a column is categorical when its GLOBAL distinct count is <= maxCategories; a rank with
        # more local distinct values already rules it out (agreed by one all-reduce)
        stats = torch.zeros(d + 2, dtype=torch.float64)
        stats[d], stats[d + 1] = float(n), float(d)
        bounded = None
        if n and X.is_cuda and d:
            # how many distinct values, up to maxCategories + 1: an early-exit hash-set pass
            # (catstats.hip small_distinct_kernel) instead of sorting every column
            from ...ops import catstats

            bounded = catstats.bounded_distinct_counts(X, max_cat)
            if bounded is not None:
                stats[:d] = torch.from_numpy(bounded.astype(np.float64))
        if n and bounded is None:
            S, _ = torch.sort(X, dim=0)
            stats[:d] = (1 + (S[1:] != S[:-1]).sum(0)).to(torch.float64).cpu()
        if dist:
            # vector length agreement over the ranks that hold rows (every rank raises together)
            dd = torch.tensor([float(d) if n else -1.0, -float(d) if n else -float(1 << 40)], dtype=torch.float64)
            dd = comm.all_reduce(dd, "max")
            if dd[0] >= 0 and float(dd[0]) != -float(dd[1]):
                raise ValueError("Feature vectors should be of equal length.")
            d = max(int(dd[0]), 0)
            loc = stats[:d].clone() if n else torch.zeros(d, dtype=torch.float64)
            red_max = comm.all_reduce(loc, "max") if d else loc
            total = comm.all_reduce_scalar(float(n), "sum")
        else:
            red_max, total = stats[:d], float(n)
        if total == 0:
            raise RuntimeError("The training set is empty.")
        cand = [c for c in range(d) if red_max[c] <= max_cat]
        maps = {}
        if cand:
            # distinct (column, value) keys over all ranks: one keyed shuffle (VectorIndexer.java's
            # per-column distinct-value aggregation)
            if n:
                Xc = X[:, cand]
                keys = torch.stack([torch.arange(len(cand), device=X.device)[None, :].expand(n, len(cand)),
                                    ds.float_keys(Xc).reshape(n, len(cand))], -1).reshape(-1, 2)
            else:
                keys = torch.zeros((0, 2), dtype=torch.int64, device=X.device)
            uk, _ = ds.global_distinct(keys)
            uk = uk.cpu()
            col, vals = uk[:, 0].numpy(), ds.keys_to_float(uk[:, 1]).numpy()
            for i, c in enumerate(cand):
                v = vals[col == i]
                if v.shape[0] <= max_cat:
                    maps[c] = _category_map(v.tolist())
        m = VectorIndexerModel().set_model_data(VectorIndexerModel.make_model_data_table([(maps,)]))
        rw_update(m, self)
        return m


# ================================================================================ KBinsDiscretizer
class KBinsDiscretizerModelParams(HasInputCol, HasOutputCol):
    pass


class KBinsDiscretizerParams(KBinsDiscretizerModelParams):
    UNIFORM = "uniform"
    QUANTILE = "quantile"
    KMEANS = "kmeans"
    STRATEGY = StringParam("strategy", "Strategy used to define the width of the bin.", "quantile",
                           ParamValidators.in_array("uniform", "quantile", "kmeans"))
    NUM_BINS = IntParam("numBins", "Number of bins to produce.", 5, ParamValidators.gt_eq(2))
    SUB_SAMPLES = IntParam("subSamples", "Maximum number of samples used to fit the model.", 200000,
                           ParamValidators.gt_eq(2))


_JAVA_DOUBLE_MIN = 4.9e-324
_JAVA_DOUBLE_MAX = 1.7976931348623157e308


def _uniform_edges(mn: float, mx: float, k: int) -> np.ndarray:
    width = (mx - mn) / k
    e = np.empty(k + 1)
    e[0] = mn
    for i in range(1, k + 1):  # sequential accumulation like the reference
        e[i] = e[i - 1] + width
    return e


def _quantile_edges(f: np.ndarray, k: int) -> np.ndarray:
    n = f.shape[0]
    width = 1.0 * n / k
    tmp = [f[int(i * width)] for i in range(k)] + [f[n - 1]]
    return np.array(sorted(set(tmp)))


def _kmeans_edges(f: np.ndarray, k: int) -> np.ndarray:
    n = f.shape[0]
    distinct = np.unique(f)
    if distinct.shape[0] <= k:
        return _uniform_edges(f[0], f[-1], k)
    width = 1.0 * n / k
    cent = np.array([f[int(i * width)] for i in range(k)], dtype=np.float64)
    old, rel, it = _JAVA_DOUBLE_MAX, _JAVA_DOUBLE_MAX, 0
    while it < 300 and rel > 1e-4:
        dist = np.abs(cent[None, :] - f[:, None])
        cid = np.argmin(dist, axis=1)  # first minimum == the reference's strict '<' scan
        loss = dist[np.arange(n), cid].sum()
        with np.errstate(invalid="ignore", divide="ignore"):
            cent = np.bincount(cid, weights=f, minlength=k) / np.bincount(cid, minlength=k)
        loss /= n
        rel = abs(loss - old)
        old = loss
        it += 1
    cent = np.sort(cent)
    e = np.empty(k + 1)
    e[0], e[k] = f[0], f[-1]
    e[1:k] = (cent[:-1] + cent[1:]) / 2
    return e


@rw.register_stage
class KBinsDiscretizerModel(ModelWithData, KBinsDiscretizerModelParams):
    """``KBinsDiscretizerModel.java``: value -> bin id (binary search, clamped to [0, #edges-2])."""

    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.kbinsdiscretizer.KBinsDiscretizerModel"
    MODEL_DATA_COLUMNS = ("binEdges",)

    @staticmethod
    def encode_record(out, row):
        out.write_int(len(row[0]))
        for e in row[0]:
            ser.write_double_array(out, np.asarray(e, dtype=np.float64))

    @staticmethod
    def decode_record(inp):
        return ([ser.read_double_array(inp) for _ in range(inp.read_int())],)

    @classmethod
    def make_model_data_table(cls, rows):
        return Table({"binEdges": [[np.asarray(e, dtype=np.float64) for e in r[0]] for r in rows]},
                     num_rows=len(rows))

    def _build_state(self, rows):
        edges = rows[0][0]
        L = max(len(e) for e in edges)
        E = torch.full((len(edges), L), float("inf"), dtype=torch.float64)
        for i, e in enumerate(edges):
            E[i, :len(e)] = torch.as_tensor(np.asarray(e, dtype=np.float64))
        lens = torch.tensor([len(e) for e in edges], dtype=torch.int64)
        return E, lens

    def transform(self, *inputs):
        t = inputs[0]
        X = _dense_matrix(t, self.get(self.INPUT_COL)).to(torch.float64)
        E, lens = self._model_state()
        E, lens = E.to(X.device), lens.to(X.device)
        if X.shape[1] != E.shape[0]:
            raise ValueError("Input vector size %d does not match the model's %d columns." % (X.shape[1], E.shape[0]))
        # batched binary search: idx = #edges <= x minus one, clamped to the last bin
        idx = torch.searchsorted(E, X.t().contiguous(), right=True) - 1
        idx = torch.minimum(idx, (lens - 2)[:, None])
        idx = torch.clamp(idx, min=0)
        return [t.with_column(self.get(self.OUTPUT_COL), idx.t().to(torch.float64).contiguous())]


@rw.register_stage
class KBinsDiscretizer(Estimator, KBinsDiscretizerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.kbinsdiscretizer.KBinsDiscretizer"

    def fit(self, *inputs):
        from ..kmeans import sample_rows

        t = inputs[0]
        X = _dense_matrix(t, self.get(self.INPUT_COL))
        strategy, k = self.get(self.STRATEGY), self.get(self.NUM_BINS)
        d = X.shape[1] if X.dim() == 2 else 0
        if strategy == self.UNIFORM:
            st = fo.column_stats(X) if X.shape[0] else None
            mn = st["min"] if st else torch.full((d,), float("inf"), dtype=torch.float64)
            mx = st["max"] if st else torch.full((d,), float("-inf"), dtype=torch.float64)
            if get_world_distributed():
                mn, mx = comm.all_reduce(mn.clone(), "min"), comm.all_reduce(mx.clone(), "max")
                n = int(comm.all_reduce_scalar(float(X.shape[0]), "sum"))
            else:
                n = X.shape[0]
            if n == 0:
                raise RuntimeError("The training set is empty.")
            mn, mx = mn.cpu().numpy(), mx.cpu().numpy()
            edges = [np.array([_JAVA_DOUBLE_MIN, _JAVA_DOUBLE_MAX]) if mn[c] == mx[c] else
                     _uniform_edges(mn[c], mx[c], k) for c in range(len(mn))]
        else:
            seed = java_string_hash(self.JAVA_CLASS_NAME)
            S = sample_rows(X, self.get(self.SUB_SAMPLES), seed)
            if S.shape[0] == 0:
                raise RuntimeError("The training set is empty.")
            edges = []
            for c in range(S.shape[1]):
                f = np.sort(S[:, c])
                if f[0] == f[-1]:
                    edges.append(np.array([_JAVA_DOUBLE_MIN, _JAVA_DOUBLE_MAX]))
                elif strategy == self.QUANTILE:
                    edges.append(_quantile_edges(f, k))
                else:
                    edges.append(_kmeans_edges(f, k))
        m = KBinsDiscretizerModel().set_model_data(KBinsDiscretizerModel.make_model_data_table([(edges,)]))
        rw_update(m, self)
        return m


# ================================================================================ Imputer
class ImputerModelParams(HasInputCols, HasOutputCols, HasRelativeError):
    MISSING_VALUE = FloatParam("missingValue", "The placeholder for the missing values. All occurrences of "
                               "missingValue will be imputed.", float("nan"))


class ImputerParams(ImputerModelParams):
    MEAN = "mean"
    MEDIAN = "median"
    MOST_FREQUENT = "most_frequent"
    STRATEGY = StringParam("strategy", "The imputation strategy.", "mean",
                           ParamValidators.in_array("mean", "median", "most_frequent"))


def _is_missing(x: torch.Tensor, missing: float) -> torch.Tensor:
    return torch.isnan(x) if math.isnan(missing) else (x == missing)


native.register_kernel_sigs({"fmlx_masked_sum_f64": [native.c_void_p, native.c_long, native.c_double, native.c_int,
                                                      native.c_void_p, native.c_void_p, native.c_void_p]})


def _valid_sum_count(x: torch.Tensor, missing: float):
    """[sum, count] of a device column's entries that are neither NaN nor ``missing`` — one pass
    of csrc/colstats.hip masked_sum_kernel (no filtered copy of the column)."""
    x = x.contiguous()
    buf = torch.empty(2 * 1024 + 2, dtype=torch.float64, device=x.device)
    native.call("fmlx_masked_sum_f64", native.ptr(x) if x.numel() else None, x.numel(), float(missing),
                int(math.isnan(missing)), native.ptr(buf), native.ptr(buf[2048:]), native.stream_ptr(x.device))
    s, c = buf[2048:].cpu().tolist()
    return [s, c]


@rw.register_stage
class ImputerModel(ModelWithData, ImputerModelParams):
    """``ImputerModel.java``: null / missingValue entries -> per-column surrogate (output double).
    Columns are read by name (the reference reads the i-th field of the row)."""

    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.imputer.ImputerModel"
    MODEL_DATA_COLUMNS = ("surrogates",)

    @staticmethod
    def encode_record(out, row):
        ser.write_map(out, _ordered_map(dict(row[0]), java_string_hash), lambda o, k: o.write_string(k),
                      lambda o, v: o.write_double(float(v)))

    @staticmethod
    def decode_record(inp):
        return (ser.read_map(inp, lambda i: i.read_string(), lambda i: i.read_double()),)

    @classmethod
    def make_model_data_table(cls, rows):
        return Table({"surrogates": [dict(r[0]) for r in rows]}, num_rows=len(rows))

    def transform(self, *inputs):
        t = inputs[0]
        sur = self.model_data_rows()[0][0]
        missing = self.get(self.MISSING_VALUE)
        res = {}
        for c, o in zip(self.get(self.INPUT_COLS), self.get(self.OUTPUT_COLS)):
            if c not in sur:
                raise ValueError("Column %s is unacceptable for the Imputer model." % c)
            x = _numeric_col(t, c).to(torch.float64)
            null = torch.isnan(x) if not isinstance(t.column(c), torch.Tensor) else torch.zeros_like(x, dtype=torch.bool)
            res[o] = torch.where(null | _is_missing(x, missing), torch.full_like(x, float(sur[c])), x)
        return [t.with_columns(res)]


@rw.register_stage
class Imputer(Estimator, ImputerParams):
    JAVA_CLASS_NAME = "org.apache.flink.ml.feature.imputer.Imputer"

    def fit(self, *inputs):
        t = inputs[0]
        cols, outs = self.get(self.INPUT_COLS), self.get(self.OUTPUT_COLS)
        if len(cols) != len(outs):
            raise ValueError("Num of input columns and output columns are inconsistent.")
        missing, strategy = self.get(self.MISSING_VALUE), self.get(self.STRATEGY)
        dist = get_world_distributed()
        xs = []
        for c in cols:
            x = _numeric_col(t, c).to(torch.float64)
            if strategy == self.MEAN and x.is_cuda:
                xs.append(x)  # (masked in the sum kernel below)
                continue
            xs.append(x[~(torch.isnan(x) | _is_missing(x, missing))])
        sur: Dict[str, float] = {}
        if strategy == self.MEAN:
            st = torch.tensor([_valid_sum_count(x, missing) if x.is_cuda else [float(x.sum()), float(x.numel())]
                               for x in xs], dtype=torch.float64)
            if dist:
                st = comm.all_reduce_sum(st)
            if st[0, 1] <= 0:
                raise RuntimeError("The training set is empty or does not contains valid data.")
            for i, c in enumerate(cols):
                sur[c] = float(st[i, 0] / st[i, 1])
        elif strategy == self.MEDIAN:
            for c, x in zip(cols, xs):
                n = int(comm.all_reduce_scalar(float(x.numel()), "sum")) if dist else x.numel()
                if n == 0:
                    raise RuntimeError("Surrogate cannot be computed. All the values in column [%s] are null, NaN or "
                                       "missingValue." % c)
                sur[c] = float(exact_quantiles(x[:, None], [0.5], self.get(self.RELATIVE_ERROR))[0, 0])
        else:
            for c, x in zip(cols, xs):
                # value counts over all ranks by a keyed shuffle of the values' bit patterns
                k, cnt = ds.global_distinct(ds.float_keys(x.reshape(-1)))
                if k.numel() == 0:
                    sur[c] = float("nan")
                    continue
                v = ds.keys_to_float(k)
                best = cnt.max()
                sur[c] = float(v[cnt == best].min())
            if all(math.isnan(v) for v in sur.values()):
                raise RuntimeError("The training set is empty or does not contains valid data.")
        m = ImputerModel().set_model_data(ImputerModel.make_model_data_table([(sur,)]))
        rw_update(m, self)
        return m
