"""Spillable record cache for replayed inputs (reference ``ITER/datacache/nonkeyed/DataCacheWriter``
/ ``DataCacheReader`` / ``DataCacheSnapshot`` and ``ITER/operator/ReplayOperator.java:62-311``).

``DataCache`` stores opaque records in the native segment store (``ops/csrc/host/datacache.cpp``):
memory segments while ``memory_budget`` allows, files under the cache directory after that (the
reference's ``iteration.data-cache.path``, here ``FMLX_DATA_CACHE_PATH`` or a temp dir).
``TableCache`` caches a stream of ``Table`` batches column by column (dense/int tensors as raw
bytes, ``SparseColumn`` as its three CSR arrays, other columns pickled — records this process wrote
itself) and replays them, optionally straight onto a GPU through pinned staging buffers with a
background prefetch thread so that disk reads and H2D copies overlap compute.

``CachedReplay`` wraps a one-pass source (iterator/generator of batches): the first pass (round 0)
tees every batch into the cache, later passes replay from it — what the reference's
``ReplayOperator`` does for ``ReplayableDataStreamList.replay`` inputs. ``finish()`` writes a
manifest so a checkpoint can reopen the cached input after a restart (``DataCacheSnapshot``).
"""
from __future__ import annotations

import ctypes
import json
import os
import pickle
import queue
import tempfile
import threading
from typing import Iterable, Iterator, List, Optional

import numpy as np
import torch

from ..ops import native
from ..table import SparseColumn, Table

_P, _I = ctypes.c_void_p, ctypes.c_int64
native.register_host_sigs({
    "fmlx_dc_open": ([ctypes.c_char_p, _I, _I], ctypes.c_void_p),
    "fmlx_dc_append": ([_P, _P, _I], ctypes.c_int64),
    "fmlx_dc_num_records": ([_P], ctypes.c_int64),
    "fmlx_dc_record_size": ([_P, _I], ctypes.c_int64),
    "fmlx_dc_read": ([_P, _I, _P], ctypes.c_int),
    "fmlx_dc_spill_all": ([_P], ctypes.c_int),
    "fmlx_dc_stats": ([_P, _P], None),
    "fmlx_dc_finish": ([_P], ctypes.c_int),
    "fmlx_dc_reopen": ([ctypes.c_char_p], ctypes.c_void_p),
    "fmlx_dc_close": ([_P, ctypes.c_int], None),
    "fmlx_dc_record_ptr": ([_P, _I], ctypes.c_void_p),
    "fmlx_dc_segment_mem": ([_P, _I, _P], ctypes.c_void_p),
})

DEFAULT_SEGMENT_BYTES = 1 << 30          # reference DataCacheWriter: segments up to 1 GB
DEFAULT_MEMORY_BUDGET = 8 << 30


def default_cache_dir() -> str:
    base = os.environ.get("FMLX_DATA_CACHE_PATH") or tempfile.gettempdir()
    return tempfile.mkdtemp(prefix="fmlx-cache-", dir=base)


class DataCache:
    """Append-only byte-record store; records are read back by index."""

    def __init__(self, path: Optional[str] = None, segment_bytes: int = DEFAULT_SEGMENT_BYTES,
                 memory_budget: int = DEFAULT_MEMORY_BUDGET, _handle=None):
        self.path = path or default_cache_dir()
        lib = native.host()
        self._h = _handle or lib.fmlx_dc_open(self.path.encode(), int(segment_bytes), int(memory_budget))
        if not self._h:
            raise RuntimeError("cannot open data cache at %s" % self.path)

    @classmethod
    def reopen(cls, path: str) -> "DataCache":
        h = native.host().fmlx_dc_reopen(path.encode())
        if not h:
            raise RuntimeError("no finished data cache at %s" % path)
        return cls(path, _handle=h)

    def append(self, data) -> int:
        if isinstance(data, (bytes, bytearray, memoryview)):
            buf = np.frombuffer(bytes(data), dtype=np.uint8)
        else:
            buf = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        idx = native.host().fmlx_dc_append(self._h, buf.ctypes.data if buf.size else None, buf.size)
        if idx < 0:
            raise RuntimeError("data cache append failed (%d)" % idx)
        return idx

    def __len__(self) -> int:
        return native.host().fmlx_dc_num_records(self._h)

    def size_of(self, i: int) -> int:
        return native.host().fmlx_dc_record_size(self._h, i)

    def read_into(self, i: int, out) -> None:
        """Copies record ``i`` into a host buffer (numpy array or CPU/pinned tensor)."""
        p = out.data_ptr() if isinstance(out, torch.Tensor) else out.ctypes.data
        rc = native.host().fmlx_dc_read(self._h, i, p)
        if rc:
            raise RuntimeError("data cache read failed (%d)" % rc)

    def read(self, i: int) -> bytes:
        out = np.empty(self.size_of(i), dtype=np.uint8)
        if out.size:
            self.read_into(i, out)
        return out.tobytes()

    def record_ptr(self, i: int) -> Optional[int]:
        """Address of record ``i`` in a memory segment (None: it lives in a file segment)."""
        p = native.host().fmlx_dc_record_ptr(self._h, i)
        return int(p) if p else None

    def memory_segments(self) -> List[tuple]:
        """(address, capacity) of every memory-resident segment."""
        out = []
        stats = self.stats()
        cap = ctypes.c_int64()
        for idx in range(stats["segments"]):
            p = native.host().fmlx_dc_segment_mem(self._h, idx, ctypes.byref(cap))
            if p:
                out.append((int(p), int(cap.value)))
        return out

    def spill(self) -> None:
        rc = native.host().fmlx_dc_spill_all(self._h)
        if rc:
            raise RuntimeError("data cache spill failed (%d)" % rc)

    def stats(self) -> dict:
        s = np.zeros(4, dtype=np.int64)
        native.host().fmlx_dc_stats(self._h, s.ctypes.data)
        return {"memory_bytes": int(s[0]), "file_bytes": int(s[1]), "segments": int(s[2]),
                "memory_segments": int(s[3])}

    def finish(self) -> None:
        rc = native.host().fmlx_dc_finish(self._h)
        if rc:
            raise RuntimeError("data cache finish failed (%d)" % rc)

    def close(self, remove: bool = True) -> None:
        if self._h:
            native.host().fmlx_dc_close(self._h, int(remove))
            self._h = None

    def __del__(self):
        try:
            self.close(remove=False)
        except Exception:
            pass


_DT = {torch.float64: "f8", torch.float32: "f4", torch.bfloat16: "bf16", torch.float16: "f2",
       torch.int64: "i8", torch.int32: "i4", torch.int16: "i2", torch.int8: "i1", torch.uint8: "u1",
       torch.bool: "b1"}
_TD = {v: k for k, v in _DT.items()}


def _tensor_bytes(t: torch.Tensor) -> np.ndarray:
    t = t.detach().contiguous().cpu()
    return t.view(torch.uint8).reshape(-1).numpy() if t.numel() else np.zeros(0, np.uint8)


class TableCache:
    """Caches ``Table`` batches; ``replay(device)`` yields them again in order."""

    def __init__(self, cache: Optional[DataCache] = None, **kw):
        self.cache = cache or DataCache(**kw)
        self.batches: List[dict] = []

    def _put_tensor(self, t: torch.Tensor) -> dict:
        return {"rec": self.cache.append(_tensor_bytes(t)), "dtype": _DT[t.dtype], "shape": list(t.shape)}

    def append(self, table: Table) -> None:
        cols = []
        for name in table.column_names:
            c = table.column(name)
            if isinstance(c, torch.Tensor):
                cols.append({"name": name, "kind": "tensor", **self._put_tensor(c)})
            elif isinstance(c, SparseColumn):
                cols.append({"name": name, "kind": "sparse", "size": c.size,
                             "parts": [self._put_tensor(p) for p in (c.indptr, c.indices, c.values)]})
            else:  # object column: pickled by this process, read back by this process only
                cols.append({"name": name, "kind": "pickle", "rec": self.cache.append(pickle.dumps(list(c)))})
        self.batches.append({"num_rows": table.num_rows, "time_col": table.time_col, "cols": cols})

    def __len__(self) -> int:
        return len(self.batches)

    def _get_tensor(self, meta: dict, device, pinned: bool) -> torch.Tensor:
        dt = _TD[meta["dtype"]]
        n = self.cache.size_of(meta["rec"])
        host = torch.empty(n, dtype=torch.uint8, pin_memory=pinned)
        if n:
            self.cache.read_into(meta["rec"], host)
        t = host.view(dt).reshape(meta["shape"])
        if device is not None and torch.device(device).type != "cpu":
            return t.to(device, non_blocking=pinned)
        return t

    def load(self, i: int, device=None) -> Table:
        b = self.batches[i]
        pinned = device is not None and torch.device(device).type == "cuda" and torch.cuda.is_available()
        cols = {}
        for c in b["cols"]:
            if c["kind"] == "tensor":
                cols[c["name"]] = self._get_tensor(c, device, pinned)
            elif c["kind"] == "sparse":
                ip, ix, vals = (self._get_tensor(p, device, pinned) for p in c["parts"])
                cols[c["name"]] = SparseColumn(ip, ix, vals, c["size"])
            else:
                cols[c["name"]] = pickle.loads(self.cache.read(c["rec"]))  # our own record
        return Table(cols, num_rows=b["num_rows"], time_col=b["time_col"])

    def replay(self, device=None, prefetch: int = 2, start: int = 0) -> Iterator[Table]:
        """Batches ``start..`` in order; with ``prefetch`` > 0 a background thread reads ahead."""
        if prefetch <= 0:
            for i in range(start, len(self.batches)):
                yield self.load(i, device)
            return
        q: "queue.Queue" = queue.Queue(maxsize=prefetch)
        stop = threading.Event()

        def work():
            try:
                for i in range(start, len(self.batches)):
                    if stop.is_set():
                        return
                    q.put(self.load(i, device))
            except BaseException as e:  # surfaced in the consumer
                q.put(e)
                return
            q.put(None)

        th = threading.Thread(target=work, daemon=True)
        th.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    return
                if isinstance(item, BaseException):
                    raise item
                yield item
        finally:
            stop.set()
            while th.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    th.join(timeout=0.05)

    def finish(self) -> None:
        """Spills to disk and writes the manifests (``DataCacheSnapshot``)."""
        self.cache.finish()
        with open(os.path.join(self.cache.path, "batches.json"), "w") as f:
            json.dump(self.batches, f)

    @classmethod
    def reopen(cls, path: str) -> "TableCache":
        tc = cls(DataCache.reopen(path))
        with open(os.path.join(path, "batches.json")) as f:
            tc.batches = json.load(f)
        return tc

    def close(self, remove: bool = True) -> None:
        self.cache.close(remove)


class CachedReplay:
    """Replayable view of a one-pass batch source: first iteration tees into a ``TableCache``,
    later iterations replay from it (``ReplayOperator`` semantics)."""

    def __init__(self, source: Iterable, device=None, **cache_kw):
        self._source = source
        self._device = device
        self._cache_kw = cache_kw
        self.cache: Optional[TableCache] = None
        self.complete = False

    def __iter__(self):
        if self.complete:
            yield from self.cache.replay(self._device)
            return
        self.cache = TableCache(**self._cache_kw)
        for batch in self._source:
            if isinstance(batch, Table):
                self.cache.append(batch)
            yield batch
        self.complete = True

    def close(self):
        if self.cache is not None:
            self.cache.close()
