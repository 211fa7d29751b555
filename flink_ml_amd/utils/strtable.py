"""Host string tables: a batch of strings as ONE array of UTF-16 code units plus int64 offsets.

High-cardinality vocabulary stages (StringIndexer, CountVectorizer, IndexToString; reference
``LIB/feature/stringindexer/StringIndexer.java:110-178``, ``StringIndexerModel.java:140-160``,
``LIB/feature/countvectorizer/CountVectorizer.java:96-160``) do per-distinct-string work: Java
``String.hashCode`` (HashMap iteration order), ``String.compareTo`` sorts, dictionary lookups and
rank merges. With 1M distinct strings a Python dict / sort per string costs seconds; here each of
those is one native batch call over the code-unit array (``ops/csrc/host/strtab.cpp``,
``javastr.cpp``), and the keyed merge across ranks moves the tables as tensors
(``parallel/datastream.reduce_strings_by_key``).
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

_SIGS = False


def _lib():
    global _SIGS
    from ..ops import native

    if not _SIGS:
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        native.register_host_sigs({
            "fmlx_str_hash64": [vp, vp, i64, vp],
            "fmlx_str_argsort": [vp, vp, i64, ctypes.c_int, vp],
            "fmlx_str_lookup": [vp, vp, i64, vp, vp, i64, vp],
            "fmlx_java_string_hashes": [vp, vp, i64, vp],
            "fmlx_hashmap_order": [vp, i64, i64, vp],
            "fmlx_str_gather": [vp, vp, vp, i64, vp, vp],
        })
        _SIGS = True
    return native.host()


class StrTable:
    """``n`` strings: ``units`` (uint16 UTF-16 code units, concatenated) and ``offs`` (int64
    [n + 1]); ``strings()`` gives the Python strings back (cached when built from them)."""

    __slots__ = ("units", "offs", "_strs")

    # _strs: the Python strings when known (a list, or an object array after a gather)
    def __init__(self, units: np.ndarray, offs: np.ndarray, strs=None):
        self.units = np.ascontiguousarray(units, dtype=np.uint16)
        self.offs = np.ascontiguousarray(offs, dtype=np.int64)
        self._strs = strs

    @staticmethod
    def from_strings(strings: Sequence[str]) -> "StrTable":
        """Raises TypeError if an element is not a str."""
        strs = strings if isinstance(strings, list) else list(strings)
        n = len(strs)
        raw = "".join(strs).encode("utf-16-le", "surrogatepass")
        units = np.frombuffer(raw, dtype=np.uint16) if raw else np.zeros(0, dtype=np.uint16)
        lens = np.fromiter(map(len, strs), dtype=np.int64, count=n)
        if int(lens.sum()) != units.shape[0]:  # astral characters take two code units
            lens = np.fromiter((len(w.encode("utf-16-le", "surrogatepass")) // 2 for w in strs), dtype=np.int64,
                               count=n)
        offs = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        return StrTable(units, offs, strs)

    def __len__(self) -> int:
        return int(self.offs.shape[0] - 1)

    def _ptrs(self):
        u = self.units if self.units.size else np.zeros(1, dtype=np.uint16)
        return u.ctypes.data, self.offs.ctypes.data, u

    def strings(self) -> List[str]:
        if isinstance(self._strs, np.ndarray):
            self._strs = self._strs.tolist()
        if self._strs is None:
            s = self.units.tobytes().decode("utf-16-le", "surrogatepass")
            if len(s) == self.units.shape[0]:  # BMP only: code units = characters
                o = self.offs.tolist()
                self._strs = [s[o[i]:o[i + 1]] for i in range(len(self))]
            else:
                b = self.units.tobytes()
                o = self.offs.tolist()
                self._strs = [b[2 * o[i]:2 * o[i + 1]].decode("utf-16-le", "surrogatepass") for i in range(len(self))]
        return self._strs

    def take(self, idx: np.ndarray) -> "StrTable":
        idx = np.ascontiguousarray(idx, dtype=np.int64)
        m = idx.shape[0]
        offs = np.zeros(m + 1, dtype=np.int64)
        if m:
            total = int((self.offs[idx + 1] - self.offs[idx]).sum())
            units = np.empty(max(total, 1), dtype=np.uint16)
            u, o, _keep = self._ptrs()
            _lib().fmlx_str_gather(u, o, idx.ctypes.data, m, units.ctypes.data, offs.ctypes.data)
            units = units[:total]
        else:
            units = np.zeros(0, dtype=np.uint16)
        strs = None
        if self._strs is not None:
            strs = _obj_array(self._strs)[idx]
        return StrTable(units, offs, strs)

    def take_strings(self, idx: np.ndarray) -> List[str]:
        """The strings at ``idx`` as a list (one object-array gather)."""
        src = self._strs if self._strs is not None else self.strings()
        return _obj_array(src)[np.asarray(idx, dtype=np.int64)].tolist()

    @staticmethod
    def concat(tables: Sequence["StrTable"]) -> "StrTable":
        units = np.concatenate([t.units for t in tables]) if tables else np.zeros(0, dtype=np.uint16)
        offs = [np.zeros(1, dtype=np.int64)]
        base = 0
        for t in tables:
            offs.append(t.offs[1:] + base)
            base += int(t.offs[-1])
        strs = None
        if tables and all(t._strs is not None for t in tables):
            strs = [s for t in tables for s in t.strings()]
        return StrTable(units, np.concatenate(offs), strs)

    # ---- native batch operations ---------------------------------------------------------
    def hash64(self) -> np.ndarray:
        """Rank-independent 64-bit content hashes (int64 view)."""
        n = len(self)
        out = np.zeros(n, dtype=np.uint64)
        if n:
            u, o, _keep = self._ptrs()
            _lib().fmlx_str_hash64(u, o, n, out.ctypes.data)
        return out.view(np.int64)

    def java_hashes(self) -> np.ndarray:
        """``String.hashCode()`` of every string (int32)."""
        n = len(self)
        out = np.zeros(n, dtype=np.int32)
        if n:
            u, o, _keep = self._ptrs()
            _lib().fmlx_java_string_hashes(u, o, n, out.ctypes.data)
        return out

    def argsort(self, descending: bool = False) -> np.ndarray:
        """Stable order by ``String.compareTo`` (UTF-16 code units)."""
        n = len(self)
        out = np.zeros(n, dtype=np.int64)
        if n:
            u, o, _keep = self._ptrs()
            _lib().fmlx_str_argsort(u, o, n, int(bool(descending)), out.ctypes.data)
        return out

    def lookup(self, queries: "StrTable") -> np.ndarray:
        """Index of the first string of this table equal to each query, −1 if absent."""
        nq = len(queries)
        out = np.full(nq, -1, dtype=np.int64)
        if nq and len(self):
            u, o, _k1 = self._ptrs()
            qu, qo, _k2 = queries._ptrs()
            _lib().fmlx_str_lookup(u, o, len(self), qu, qo, nq, out.ctypes.data)
        return out

    def first_of_equal(self) -> np.ndarray:
        """For every string, the index of its first occurrence in this table."""
        return self.lookup(self)


def _obj_array(strs) -> np.ndarray:
    if isinstance(strs, np.ndarray):
        return strs
    a = np.empty(len(strs), dtype=object)
    a[:] = strs
    return a


def hashmap_order_from_hashes(h: np.ndarray, initial_capacity: int = 16) -> np.ndarray:
    """Iteration order of a ``java.util.HashMap`` filled with keys of Java hashes ``h`` in index
    order (no treeified bins; same rule as ``utils.java.java_hashmap_order``): a stable sort by
    the final table's bucket."""
    n = int(h.shape[0])
    cap = 1
    while cap < initial_capacity:
        cap <<= 1
    cap = max(cap, 1)
    while n > cap * 0.75:
        cap *= 2
    hh = np.ascontiguousarray(h, dtype=np.int32)
    out = np.zeros(n, dtype=np.int64)
    if n:
        _lib().fmlx_hashmap_order(hh.ctypes.data, n, cap, out.ctypes.data)
    return out
