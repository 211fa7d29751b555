"""Greenwald–Khanna ε-approximate quantile summary (reference
``LIB/common/util/QuantileSummary.java:39-414``), for users that build sketches themselves.

The library's own stages (RobustScaler, Imputer median, KBinsDiscretizer) do not use it: on the
GPU they compute exact order statistics by distributed radix select (``ops/quantile.py``), which
answers the same queries with zero rank error and without shipping sketches between ranks.

The summary is immutable in the reference's style (``insert``/``compress``/``merge`` return the
summary to keep using). Samples are (value, g, delta) numpy arrays; the O(n) passes — head-buffer
insertion, compression, merge and query — run in native C++ (``ops/csrc/host/gk.cpp``).
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Union

import numpy as np

from ..ops import native

_P = ctypes.c_void_p
_I = ctypes.c_int64
native.register_host_sigs({
    "fmlx_gk_insert": ([_P, _P, _P, _I, _P, _I, _I, _P, _P, _P], ctypes.c_int64),
    "fmlx_gk_compress": ([_P, _P, _P, _I, ctypes.c_double, _P, _P, _P], ctypes.c_int64),
    "fmlx_gk_merge": ([_P, _P, _P, _I, _P, _P, _P, _I, _I, _I, _P, _P, _P], ctypes.c_int64),
    "fmlx_gk_query": ([_P, _P, _P, _I, _I, ctypes.c_double, _P, _I, _P], None),
})

DEFAULT_HEAD_SIZE = 50000
DEFAULT_COMPRESS_THRESHOLD = 10000


def _p(a: np.ndarray):
    return a.ctypes.data if a.size else None


def _empty(n=0):
    return np.empty(n, np.float64), np.empty(n, np.int64), np.empty(n, np.int64)


class QuantileSummary:
    def __init__(self, relative_error: float, compress_threshold: int = DEFAULT_COMPRESS_THRESHOLD,
                 _samples=None, _count: int = 0, _compressed: bool = False):
        if not 0 <= relative_error <= 1:
            raise ValueError("An appropriate relative error must be in the range [0, 1].")
        if compress_threshold <= 0:
            raise ValueError("An compress threshold must greater than 0.")
        self.relative_error = float(relative_error)
        self.compress_threshold = int(compress_threshold)
        self._v, self._g, self._d = _samples if _samples is not None else _empty()
        self.count = int(_count)
        self.compressed = bool(_compressed)
        self._head: List[float] = []

    # ------------------------------------------------------------------ reference API
    def insert(self, item: float) -> "QuantileSummary":
        self._head.append(float(item))
        self.compressed = False
        if len(self._head) >= DEFAULT_HEAD_SIZE:
            res = self._insert_head_buffer()
            return res.compress() if res._v.size >= self.compress_threshold else res
        return self

    def insert_all(self, items) -> "QuantileSummary":
        """Batch insert with the same result as inserting the items one by one."""
        s = self
        arr = np.asarray(items, dtype=np.float64).reshape(-1)
        pos = 0
        while pos < arr.size:
            room = DEFAULT_HEAD_SIZE - len(s._head)
            take = arr[pos:pos + room]
            pos += take.size
            if take.size < room:
                s._head.extend(take.tolist())
                s.compressed = False
                break
            s._head.extend(take[:-1].tolist())
            s = s.insert(float(take[-1]))
        return s

    def compress(self) -> "QuantileSummary":
        if self.compressed:
            return self
        ins = self._insert_head_buffer()
        v, g, d = _compress(ins._v, ins._g, ins._d, 2 * self.relative_error * ins.count)
        return QuantileSummary(self.relative_error, self.compress_threshold, (v, g, d), ins.count, True)

    def merge(self, other: "QuantileSummary") -> "QuantileSummary":
        if self._head:
            raise RuntimeError("Current buffer needs to be compressed before merge.")
        if other._head:
            raise RuntimeError("Other buffer needs to be compressed before merge.")
        if other.count == 0:
            return self._shallow_copy()
        if self.count == 0:
            return other._shallow_copy()
        err = max(self.relative_error, other.relative_error)
        total = self.count + other.count
        add_self = int(np.floor(2 * other.relative_error * other.count))
        add_other = int(np.floor(2 * self.relative_error * self.count))
        n = self._v.size + other._v.size
        ov, og, od = _empty(n)
        m = native.host().fmlx_gk_merge(_p(self._v), _p(self._g), _p(self._d), self._v.size, _p(other._v),
                                        _p(other._g), _p(other._d), other._v.size, add_self, add_other,
                                        _p(ov), _p(og), _p(od))
        v, g, d = _compress(ov[:m], og[:m], od[:m], 2 * err * total)
        return QuantileSummary(err, self.compress_threshold, (v, g, d), total, True)

    def query(self, percentiles: Union[float, Sequence[float]]):
        single = np.isscalar(percentiles)
        ps = np.atleast_1d(np.asarray(percentiles, dtype=np.float64))
        if ((ps < 0) | (ps > 1)).any():
            raise RuntimeError("percentile should be in the range [0.0, 1.0].")
        if self._head:
            raise RuntimeError("Cannot operate on an uncompressed summary, call compress() first.")
        if self._v.size == 0:
            raise RuntimeError("Cannot query percentiles without any records inserted.")
        order = np.argsort(ps, kind="stable")
        sorted_ps = np.ascontiguousarray(ps[order])
        res = np.empty(ps.size, np.float64)
        native.host().fmlx_gk_query(_p(self._v), _p(self._g), _p(self._d), self._v.size, self.count,
                                    self.relative_error, _p(sorted_ps), ps.size, _p(res))
        out = np.empty_like(res)
        out[order] = res
        return float(out[0]) if single else out

    def is_empty(self) -> bool:
        return not self._head and self._v.size == 0

    def get_relative_error(self) -> float:
        return self.relative_error

    # ------------------------------------------------------------------ internals
    def _insert_head_buffer(self) -> "QuantileSummary":
        if not self._head:
            return self
        h = np.sort(np.asarray(self._head, dtype=np.float64))
        n = self._v.size + h.size
        ov, og, od = _empty(n)
        delta = int(np.floor(2.0 * self.relative_error * self.count))
        m = native.host().fmlx_gk_insert(_p(self._v), _p(self._g), _p(self._d), self._v.size, _p(h), h.size,
                                         delta, _p(ov), _p(og), _p(od))
        assert m == n
        return QuantileSummary(self.relative_error, self.compress_threshold, (ov, og, od), self.count + h.size, False)

    def _shallow_copy(self) -> "QuantileSummary":
        return QuantileSummary(self.relative_error, self.compress_threshold, (self._v, self._g, self._d),
                               self.count, self.compressed)

    @property
    def samples(self):
        """(values, g, delta) arrays of the compressed summary."""
        return self._v, self._g, self._d

    def __eq__(self, other) -> bool:
        return (isinstance(other, QuantileSummary) and self.relative_error == other.relative_error
                and self.count == other.count and np.array_equal(self._v, other._v)
                and np.array_equal(self._g, other._g) and np.array_equal(self._d, other._d)
                and self._head == other._head)

    __hash__ = None


def _compress(v, g, d, thr):
    v, g, d = (np.ascontiguousarray(a) for a in (v, g, d))
    ov, og, od = _empty(v.size)
    m = native.host().fmlx_gk_compress(_p(v), _p(g), _p(d), v.size, float(thr), _p(ov), _p(og), _p(od))
    return ov[:m].copy(), og[:m].copy(), od[:m].copy()
