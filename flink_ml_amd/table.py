"""Columnar, device-resident tables.

Replaces the reference's Flink ``Table``/``DataStream<Row>``: instead of a
stream of boxed ``Row`` objects, a ``Table`` is an ordered set of named columns, each one of

* ``torch.Tensor`` of rank 1 — a numeric scalar column (double/long/int/bool),
* ``torch.Tensor`` of rank 2 — a *dense vector* column, row i = vector i (this is the form
  the HIP kernels consume; it stays in HBM between pipeline stages),
* ``SparseColumn`` — a CSR batch of sparse vectors (indptr/indices/values tensors),
* ``list`` — host objects (strings, string arrays, mixed vectors, anything else).

In an SPMD job every rank holds *its own partition* of each table (the analogue of a
Flink subtask's slice of a stream); collectives in ``flink_ml_amd.parallel`` combine them.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional, Sequence

import numpy as np
import torch

from .linalg.vectors import DenseVector, SparseVector, Vector


class SparseColumn:
    """CSR batch of sparse vectors of a common logical size."""

    __slots__ = ("indptr", "indices", "values", "size")

    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor, values: torch.Tensor, size: int):
        self.indptr = indptr
        self.indices = indices
        self.values = values
        self.size = int(size)

    def __len__(self):
        return int(self.indptr.shape[0]) - 1

    @property
    def device(self):
        return self.values.device

    def to(self, device=None, dtype=None) -> "SparseColumn":
        return SparseColumn(
            self.indptr.to(device) if device is not None else self.indptr,
            self.indices.to(device) if device is not None else self.indices,
            self.values.to(device=device, dtype=dtype) if (device is not None or dtype is not None) else self.values,
            self.size,
        )

    @staticmethod
    def from_vectors(vectors: Sequence[Vector], size: int = None) -> "SparseColumn":
        n = len(vectors)
        if size is None:
            size = max((v.size() for v in vectors), default=0)
        lens = np.zeros(n + 1, dtype=np.int64)
        idx_parts, val_parts = [], []
        for i, v in enumerate(vectors):
            if isinstance(v, SparseVector):
                ii, vv = v.indices, v.values
            else:
                arr = v.to_array()
                ii = np.nonzero(arr)[0].astype(np.int32)
                vv = arr[ii]
            lens[i + 1] = ii.shape[0]
            idx_parts.append(ii)
            val_parts.append(vv)
        indptr = np.cumsum(lens)
        indices = np.concatenate(idx_parts).astype(np.int32) if idx_parts else np.zeros(0, np.int32)
        values = np.concatenate(val_parts).astype(np.float64) if val_parts else np.zeros(0, np.float64)
        return SparseColumn(torch.from_numpy(indptr), torch.from_numpy(indices), torch.from_numpy(values), size)

    def row(self, i: int) -> SparseVector:
        s, e = int(self.indptr[i]), int(self.indptr[i + 1])
        return SparseVector(self.size, self.indices[s:e].cpu().numpy(), self.values[s:e].double().cpu().numpy())

    def to_dense(self, dtype=torch.float64, device=None) -> torch.Tensor:
        n = len(self)
        device = device if device is not None else self.values.device
        out = torch.zeros((n, self.size), dtype=dtype, device=device)
        if self.values.numel():
            counts = (self.indptr[1:] - self.indptr[:-1]).to(device)
            rows = torch.repeat_interleave(torch.arange(n, device=device), counts)
            out[rows, self.indices.to(device).long()] = self.values.to(device=device, dtype=dtype)
        return out

    @staticmethod
    def from_dense(X: torch.Tensor) -> "SparseColumn":
        """Nonzero entries of a dense [n, d] tensor as CSR, on X's device (``DenseVector.toSparse``)."""
        nzr, nzc = torch.nonzero(X, as_tuple=True)
        indptr = torch.zeros(X.shape[0] + 1, dtype=torch.int64, device=X.device)
        indptr[1:] = torch.cumsum(torch.bincount(nzr, minlength=X.shape[0]), 0)
        return SparseColumn(indptr, nzc.to(torch.int32), X[nzr, nzc].to(torch.float64), int(X.shape[1]))

    @staticmethod
    def concat(parts: Sequence["SparseColumn"]) -> "SparseColumn":
        """Row-wise concatenation (sizes must agree); result on the first part's device."""
        parts = list(parts)
        dev = parts[0].values.device
        ptrs, off = [torch.zeros(1, dtype=torch.int64, device=dev)], 0
        for p in parts:
            ptrs.append(p.indptr[1:].to(dev).long() + off)
            off += int(p.indptr[-1])
        return SparseColumn(torch.cat(ptrs), torch.cat([p.indices.to(dev) for p in parts]),
                            torch.cat([p.values.to(dev) for p in parts]), max(p.size for p in parts))

    def slice(self, start: int, end: int) -> "SparseColumn":
        """Rows [start, end) without copying: views of indices/values and a rebased indptr."""
        n = len(self)
        start, end = max(0, min(start, n)), max(0, min(end, n))
        end = max(end, start)
        bounds = self.indptr[[start, end]].cpu()
        s, e = int(bounds[0]), int(bounds[1])
        return SparseColumn(self.indptr[start:end + 1] - s, self.indices[s:e], self.values[s:e], self.size)

    def take(self, idx: torch.Tensor) -> "SparseColumn":
        idx = idx.cpu().long()
        vecs = [self.row(int(i)) for i in idx]
        return SparseColumn.from_vectors(vecs, self.size)


class StringArrayColumn:
    """Ragged arrays of dictionary-encoded strings: row i is
    ``[vocab[c] for c in codes[offsets[i]:offsets[i + 1]]]``.

    ``offsets``/``codes`` are tensors (HBM-resident on the GPU), ``vocab`` a host list of the
    distinct strings. String-array stages (StopWordsRemover, CountVectorizer, HashingTF) work on
    the codes with device kernels; everything else sees a sequence of Python lists (rows are
    materialised on demand), so the column is a drop-in for a list-of-lists column.
    """

    __slots__ = ("offsets", "codes", "vocab")

    def __init__(self, offsets: torch.Tensor, codes: torch.Tensor, vocab: Sequence[Optional[str]]):
        self.offsets = offsets
        self.codes = codes
        self.vocab = list(vocab)

    @staticmethod
    def from_dense_codes(codes: torch.Tensor, vocab) -> "StringArrayColumn":
        """[n, a] code matrix (every row holds a strings)."""
        n, a = codes.shape
        off = torch.arange(0, (n + 1) * a, a, dtype=torch.int64, device=codes.device)[: n + 1]
        return StringArrayColumn(off, codes.reshape(-1).to(torch.int32), vocab)

    @staticmethod
    def from_lists(rows: Sequence[Sequence[Optional[str]]]) -> "StringArrayColumn":
        index, vocab, codes, off = {}, [], [], [0]
        for r in rows:
            for w in r:
                c = index.get(w)
                if c is None:
                    c = index[w] = len(vocab)
                    vocab.append(w)
                codes.append(c)
            off.append(len(codes))
        return StringArrayColumn(torch.tensor(off, dtype=torch.int64), torch.tensor(codes, dtype=torch.int32), vocab)

    def __len__(self):
        return int(self.offsets.shape[0]) - 1

    @property
    def device(self):
        return self.codes.device

    def row_lengths(self) -> torch.Tensor:
        return self.offsets[1:] - self.offsets[:-1]

    def row_ids(self) -> torch.Tensor:
        """Row index of every code (int64, on the codes' device)."""
        n = len(self)
        return torch.repeat_interleave(torch.arange(n, device=self.codes.device), self.row_lengths().to(self.codes.device),
                                       output_size=int(self.codes.shape[0]))

    def to(self, device=None) -> "StringArrayColumn":
        if device is None:
            return self
        return StringArrayColumn(self.offsets.to(device), self.codes.to(device), self.vocab)

    def to_lists(self) -> List[List[Optional[str]]]:
        off = self.offsets.cpu().numpy()
        words = np.empty(len(self.vocab), dtype=object)
        words[:] = self.vocab
        flat = words[self.codes.cpu().numpy().astype(np.int64)].tolist()
        return [flat[off[i] - off[0]:off[i + 1] - off[0]] for i in range(len(self))]

    def __iter__(self):
        return iter(self.to_lists())

    def __getitem__(self, i):
        if isinstance(i, slice):
            start, stop, step = i.indices(len(self))
            if step != 1:
                return self.to_lists()[i]
            stop = max(stop, start)
            b = self.offsets[[start, stop]].cpu()
            # self-consistent slice: offsets rebased onto the cut codes (offsets[0] == 0), so a
            # slice of a slice and row indexing of a slice read the right codes
            off = self.offsets[start:stop + 1]
            return StringArrayColumn(off - off[:1], self.codes[int(b[0]):int(b[1])], self.vocab)
        i = int(i)
        if i < 0:
            i += len(self)
        b = self.offsets[[i, i + 1]].cpu()
        return [self.vocab[c] for c in self.codes[int(b[0]):int(b[1])].cpu().tolist()]

    def rebased(self) -> "StringArrayColumn":
        """The same rows with offsets starting at 0 (a no-op for slices, which are rebased; kept for
        columns built with an offset base)."""
        o0 = self.offsets[:1]
        return StringArrayColumn(self.offsets - o0, self.codes, self.vocab)


def first_occurrence(codes: torch.Tensor, V: int) -> torch.Tensor:
    """Position of the first occurrence of every code in ``codes`` (``len(codes)`` if absent).
    A scatter-min over a geometrically growing prefix: codes usually all appear early, so the
    min does not run over (and contend on) the whole column."""
    codes = codes.long()
    N = int(codes.shape[0])
    present = torch.nonzero(torch.bincount(codes, minlength=V) > 0).reshape(-1)
    first = torch.full((V,), N, dtype=torch.int64, device=codes.device)
    s0, step = 0, 1 << 20
    while s0 < N:
        e0 = min(N, s0 + step)
        first.scatter_reduce_(0, codes[s0:e0], torch.arange(s0, e0, device=codes.device), reduce="amin")
        if not bool((first[present] == N).any()):
            break
        s0, step = e0, step * 4
    return first


class StringColumn:
    """Dictionary-encoded strings: row i is ``vocab[codes[i]]`` (int32 codes on the device, the
    distinct strings on the host). Stages that act per string (Tokenizer, RegexTokenizer,
    StringIndexer) do their work once per distinct string and gather by code; everything else sees
    a sequence of Python strings."""

    __slots__ = ("codes", "vocab")

    def __init__(self, codes: torch.Tensor, vocab: Sequence[Optional[str]]):
        self.codes = codes
        self.vocab = list(vocab)

    @staticmethod
    def from_list(values: Sequence[Optional[str]]) -> "StringColumn":
        index, vocab, codes = {}, [], []
        for w in values:
            c = index.get(w)
            if c is None:
                c = index[w] = len(vocab)
                vocab.append(w)
            codes.append(c)
        return StringColumn(torch.tensor(codes, dtype=torch.int32), vocab)

    def __len__(self):
        return int(self.codes.shape[0])

    @property
    def device(self):
        return self.codes.device

    def to(self, device=None) -> "StringColumn":
        return self if device is None else StringColumn(self.codes.to(device), self.vocab)

    def to_list(self) -> List[Optional[str]]:
        words = np.empty(len(self.vocab), dtype=object)
        words[:] = self.vocab
        return words[self.codes.cpu().numpy().astype(np.int64)].tolist()

    def __iter__(self):
        return iter(self.to_list())

    def __getitem__(self, i):
        if isinstance(i, slice):
            return StringColumn(self.codes[i], self.vocab)
        return self.vocab[int(self.codes[int(i)])]

    def take(self, idx: torch.Tensor) -> "StringColumn":
        return StringColumn(self.codes[idx.to(self.codes.device)], self.vocab)


Column = Any  # torch.Tensor | SparseColumn | StringArrayColumn | StringColumn | list


def _col_len(col) -> int:
    if isinstance(col, torch.Tensor):
        return int(col.shape[0])
    return len(col)


def compact_column(values: List[Any]) -> Column:
    """Chooses the columnar representation for a list of row values."""
    if len(values) == 0:
        return values
    first = values[0]
    if all(isinstance(v, DenseVector) for v in values):
        d = first.size()
        if all(v.size() == d for v in values):
            return torch.from_numpy(np.stack([v.values for v in values]).astype(np.float64)) if d > 0 else values
        return list(values)
    if all(isinstance(v, SparseVector) for v in values):
        d = first.size()
        if all(v.size() == d for v in values):
            return SparseColumn.from_vectors(values, d)
        return list(values)
    if all(isinstance(v, (bool, np.bool_)) for v in values):
        return torch.tensor([bool(v) for v in values], dtype=torch.bool)
    if all(isinstance(v, (int, np.integer)) and not isinstance(v, (bool, np.bool_)) for v in values):
        return torch.tensor([int(v) for v in values], dtype=torch.int64)
    if all(isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, (bool, np.bool_)) for v in values):
        return torch.tensor([float(v) for v in values], dtype=torch.float64)
    return list(values)


def _row_value(col, i: int):
    if isinstance(col, torch.Tensor):
        if col.dim() == 2:
            return DenseVector(col[i].double().cpu().numpy())
        if col.dim() == 3:  # DenseVector[] per row (e.g. LSH hash signatures)
            return [DenseVector(r) for r in col[i].double().cpu().numpy()]
        v = col[i].item()
        return v
    if isinstance(col, SparseColumn):
        return col.row(i)
    return col[i]


class Table:
    """An ordered mapping of column name → column (see module docstring)."""

    def __init__(self, columns: Optional[Dict[str, Column]] = None, num_rows: Optional[int] = None,
                 time_col: Optional[str] = None):
        self._cols: Dict[str, Column] = dict(columns or {})
        # event-time attribute (the analogue of a Flink rowtime column with a watermark): time
        # windows cut on it; it survives column-preserving transformations
        self.time_col = time_col if time_col in self._cols else None
        # True when every rank holds the same rows (model data, test statistics, metrics) rather
        # than its own partition
        self.replicated = False
        if num_rows is None:
            num_rows = _col_len(next(iter(self._cols.values()))) if self._cols else 0
        self._n = int(num_rows)
        for name, c in self._cols.items():
            if _col_len(c) != self._n:
                raise ValueError("Column %s has %d rows, expected %d" % (name, _col_len(c), self._n))

    # -- construction ------------------------------------------------------------------------
    @staticmethod
    def from_rows(rows: Iterable[Sequence[Any]], names: Sequence[str]) -> "Table":
        rows = [tuple(r) for r in rows]
        cols = {}
        for j, name in enumerate(names):
            cols[name] = compact_column([r[j] for r in rows])
        return Table(cols, num_rows=len(rows))

    @staticmethod
    def from_columns(**cols) -> "Table":
        return Table(cols)

    @staticmethod
    def concat(tables: Sequence["Table"]) -> "Table":
        tables = [t for t in tables if t is not None]
        if not tables:
            return Table()
        names = tables[0].column_names
        out = {}
        for name in names:
            parts = [t.column(name) for t in tables]
            if all(isinstance(p, torch.Tensor) for p in parts) and len({(p.dim(), tuple(p.shape[1:])) for p in parts}) == 1:
                dev = parts[0].device
                out[name] = torch.cat([p.to(dev) for p in parts], dim=0)
            elif all(isinstance(p, SparseColumn) for p in parts) and len({p.size for p in parts}) == 1:
                out[name] = SparseColumn.concat(parts)
            else:
                rows = []
                for t in tables:
                    rows.extend(t.get_list(name))
                out[name] = compact_column(rows)
        return Table(out, num_rows=sum(t.num_rows for t in tables), time_col=tables[0].time_col)

    # -- introspection -----------------------------------------------------------------------
    @property
    def column_names(self) -> List[str]:
        return list(self._cols.keys())

    def get_column_names(self) -> List[str]:
        return self.column_names

    @property
    def num_rows(self) -> int:
        return self._n

    def __len__(self) -> int:
        return self._n

    def has_column(self, name: str) -> bool:
        return name in self._cols

    def column(self, name: str) -> Column:
        if name not in self._cols:
            raise KeyError("Column %s not found in table with columns %s" % (name, self.column_names))
        return self._cols[name]

    def __getitem__(self, name: str) -> Column:
        return self.column(name)

    # -- row-level access --------------------------------------------------------------------
    def get_list(self, name: str) -> List[Any]:
        col = self.column(name)
        if isinstance(col, list):
            return col
        if isinstance(col, StringArrayColumn):
            return col.to_lists()
        if isinstance(col, StringColumn):
            return col.to_list()
        return [_row_value(col, i) for i in range(self._n)]

    def rows(self) -> List[tuple]:
        lists = [self.get_list(n) for n in self.column_names]
        return [tuple(l[i] for l in lists) for i in range(self._n)]

    to_rows = rows

    # -- typed column accessors used by kernels ---------------------------------------------
    def vectors_as_matrix(self, name: str, dtype=torch.float64, device=None) -> torch.Tensor:
        """Dense [n, d] tensor for a vector column (dense, sparse or list-of-vectors)."""
        col = self.column(name)
        if isinstance(col, torch.Tensor):
            if col.dim() == 1:
                col = col.reshape(-1, 1)
            return col.to(device=device if device is not None else col.device, dtype=dtype)
        if isinstance(col, SparseColumn):
            return col.to_dense(dtype=dtype, device=device)
        if self._n == 0:
            return torch.zeros((0, 0), dtype=dtype, device=device)
        vecs = [v if isinstance(v, Vector) else DenseVector(v) for v in col]
        d = max(v.size() for v in vecs)
        arr = np.zeros((len(vecs), d), dtype=np.float64)
        for i, v in enumerate(vecs):
            if isinstance(v, SparseVector):
                arr[i, v.indices] = v.values
            else:
                arr[i, : v.size()] = v.values
        return torch.from_numpy(arr).to(device=device, dtype=dtype)

    def scalars(self, name: str, dtype=torch.float64, device=None) -> torch.Tensor:
        col = self.column(name)
        if isinstance(col, torch.Tensor):
            if col.dim() != 1:
                raise ValueError("Column %s is not a scalar column" % name)
            return col.to(device=device if device is not None else col.device, dtype=dtype)
        return torch.tensor([float(v) for v in col], dtype=dtype, device=device)

    def vector_size(self, name: str) -> int:
        col = self.column(name)
        if isinstance(col, torch.Tensor):
            return int(col.shape[1]) if col.dim() == 2 else 1
        if isinstance(col, SparseColumn):
            return col.size
        return max((v.size() for v in col), default=0)

    def is_sparse(self, name: str) -> bool:
        col = self.column(name)
        if isinstance(col, SparseColumn):
            return True
        if isinstance(col, list):
            return any(isinstance(v, SparseVector) for v in col)
        return False

    # -- transformations (all return new tables; columns are shared, not copied) -------------
    def with_column(self, name: str, col: Column) -> "Table":
        cols = dict(self._cols)
        cols[name] = col
        return Table(cols, num_rows=self._n, time_col=self.time_col)

    def with_columns(self, mapping: Dict[str, Column]) -> "Table":
        cols = dict(self._cols)
        cols.update(mapping)
        return Table(cols, num_rows=self._n, time_col=self.time_col)

    def select(self, *names: str) -> "Table":
        if len(names) == 1 and isinstance(names[0], (list, tuple)):
            names = tuple(names[0])
        return Table({n: self.column(n) for n in names}, num_rows=self._n, time_col=self.time_col)

    def drop(self, *names: str) -> "Table":
        return Table({k: v for k, v in self._cols.items() if k not in names}, num_rows=self._n, time_col=self.time_col)

    def rename(self, mapping: Dict[str, str]) -> "Table":
        return Table({mapping.get(k, k): v for k, v in self._cols.items()}, num_rows=self._n,
                     time_col=mapping.get(self.time_col, self.time_col))

    def as_replicated(self) -> "Table":
        self.replicated = True
        return self

    def with_time_column(self, name: str) -> "Table":
        """Marks ``name`` (epoch milliseconds) as the event-time attribute for time windows."""
        if name not in self._cols:
            raise KeyError(name)
        return Table(dict(self._cols), num_rows=self._n, time_col=name)

    def take(self, idx) -> "Table":
        if isinstance(idx, torch.Tensor) and idx.dtype == torch.bool:
            idx = torch.nonzero(idx.cpu(), as_tuple=False).reshape(-1)
        idx_t = torch.as_tensor(idx, dtype=torch.long).cpu()
        cols = {}
        for k, c in self._cols.items():
            if isinstance(c, torch.Tensor):
                cols[k] = c[idx_t.to(c.device)]
            elif isinstance(c, SparseColumn):
                cols[k] = c.take(idx_t)
            elif isinstance(c, StringColumn):
                cols[k] = c.take(idx_t)
            elif isinstance(c, StringArrayColumn):
                lists = c.to_lists()
                cols[k] = [lists[int(i)] for i in idx_t]
            else:
                cols[k] = [c[int(i)] for i in idx_t]
        return Table(cols, num_rows=int(idx_t.shape[0]), time_col=self.time_col)

    def slice(self, start: int, end: int) -> "Table":
        """Rows [start, end): tensor columns are views (no gather, no HBM traffic), so streaming a
        device-resident table in mini-batches costs nothing per batch."""
        start = max(0, min(start, self._n))
        end = max(start, min(end, self._n))
        cols = {}
        for k, c in self._cols.items():
            if isinstance(c, (torch.Tensor, SparseColumn)):
                cols[k] = c[start:end] if isinstance(c, torch.Tensor) else c.slice(start, end)
            else:
                cols[k] = c[start:end]
        return Table(cols, num_rows=end - start, time_col=self.time_col)

    def filter(self, mask) -> "Table":
        return self.take(torch.as_tensor(mask, dtype=torch.bool))

    def to(self, device) -> "Table":
        cols = {}
        for k, c in self._cols.items():
            if isinstance(c, (torch.Tensor, SparseColumn, StringArrayColumn, StringColumn)):
                cols[k] = c.to(device)
            else:
                cols[k] = c
        return Table(cols, num_rows=self._n, time_col=self.time_col)

    def partition(self, rank: int, world: int) -> "Table":
        """Round-robin partition, the analogue of Flink's ``rebalance()``."""
        return self.take(torch.arange(rank, self._n, world))

    def __repr__(self):
        return "Table(rows=%d, columns=%s)" % (self._n, self.column_names)
