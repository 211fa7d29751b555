"""Unbounded inputs: streams of mini-batch tables.

The reference's online algorithms consume unbounded ``DataStream``s. Here an
unbounded table is a ``StreamTable``: an iterator of ``Table`` mini-batches with

* ``InMemorySource`` — a thread-safe queue source the test-suite (and applications) push batches
  into while consumers run (the analogue of the reference tests' ``InMemorySourceFunction``);
* ``StreamTable.from_table`` — replay a bounded table as a stream of fixed-size batches;
* device prefetch — the next batch's host→HBM copy is issued on a side HIP stream while the
  current batch is being processed (pinned host staging), so ingestion overlaps compute;
* ``rebatch`` — regroup arbitrary arrival sizes into fixed global mini-batches, split across
  ranks exactly like ``DataStreamUtils.generateBatchData`` (remainder to low ranks).
"""
from __future__ import annotations

import queue
import threading
from typing import Callable, Iterable, Iterator, List, Optional

import torch

from .parallel.context import get_context
from .table import SparseColumn, Table


class _End:
    pass


END = _End()


class InMemorySource:
    """Queue-backed unbounded source; ``close()`` ends the stream."""

    def __init__(self):
        self._q: "queue.Queue" = queue.Queue()
        self._closed = False

    def add(self, table: Table) -> None:
        self._q.put(table)

    def add_rows(self, rows, names) -> None:
        self._q.put(Table.from_rows(rows, names))

    def close(self) -> None:
        self._closed = True
        self._q.put(END)

    def poll(self, timeout: Optional[float] = None):
        """Next batch, or None when nothing is available within ``timeout`` (non-blocking if 0)."""
        try:
            item = self._q.get(block=timeout is None or timeout > 0, timeout=timeout if timeout else None)
        except queue.Empty:
            return None
        return item

    def __iter__(self):
        while True:
            item = self._q.get()
            if item is END:
                return
            yield item


class StreamTable:
    """An (possibly unbounded) sequence of Table mini-batches."""

    def __init__(self, source: Iterable, names: Optional[List[str]] = None):
        self._source = source
        self.names = names

    # -- constructors ---------------------------------------------------------------------------
    @staticmethod
    def from_table(table: Table, batch_rows: int) -> "StreamTable":
        def gen():
            for s in range(0, table.num_rows, batch_rows):
                yield table.slice(s, s + batch_rows)
        return StreamTable(gen(), table.column_names)

    @staticmethod
    def from_tables(tables: Iterable[Table]) -> "StreamTable":
        return StreamTable(iter(tables))

    @staticmethod
    def from_source(src: InMemorySource) -> "StreamTable":
        return StreamTable(src)

    def __iter__(self) -> Iterator[Table]:
        return iter(self._source)

    # -- transformations ------------------------------------------------------------------------
    def map(self, fn: Callable[[Table], Table]) -> "StreamTable":
        return StreamTable((fn(t) for t in self), None)

    def to_device(self, device=None) -> "StreamTable":
        """Asynchronous H2D prefetch of the next batch on a side stream."""
        dev = device or get_context().device
        if dev.type != "cuda":
            return self
        return StreamTable(_prefetch(iter(self), dev), self.names)

    def rebatch(self, global_batch_size: int) -> "StreamTable":
        return StreamTable(_rebatch(iter(self), global_batch_size), self.names)


def _prefetch(it: Iterator[Table], dev) -> Iterator[Table]:
    """Copies batch k+1 host→device on a side stream while batch k is consumed. The device
    copies are allocated on the side stream, so each is marked used by the consumer stream
    (``record_stream``) before it is handed out: the caching allocator then cannot give its
    blocks to a later side-stream copy while consumer kernels still read them."""
    from .utils import streamcheck

    from .utils import graphs

    side = graphs.aux_stream(dev, "h2d-prefetch")
    nxt = None
    check = streamcheck.enabled()  # FMLX_STREAM_CHECK=1: verify every hand-off (slow)
    count = [0]

    def host_cols(t):
        return any((isinstance(c, torch.Tensor) and c.device.type == "cpu")
                   or (isinstance(c, SparseColumn) and c.values.device.type == "cpu") for c in t._cols.values())

    def issue(t):
        if t is None:
            return None
        if not host_cols(t):
            # already device-resident (zero-copy slices of an HBM table): nothing to copy, no
            # side-stream hand-off — the event / stream bookkeeping cost ~20 µs per batch
            return t, None, (), None
        fresh, pairs = [], []
        with torch.cuda.stream(side):
            cols = {}
            for k, c in t._cols.items():
                if isinstance(c, torch.Tensor) and c.device.type == "cpu":
                    cols[k] = c.pin_memory().to(dev, non_blocking=True)
                    fresh.append(cols[k])
                    pairs.append((k, c, cols[k]))
                elif isinstance(c, SparseColumn) and c.values.device.type == "cpu":
                    cols[k] = c.to(dev)
                    fresh.extend([cols[k].indptr, cols[k].indices, cols[k].values])
                    pairs.extend([(k + ".indptr", c.indptr, cols[k].indptr), (k + ".indices", c.indices, cols[k].indices),
                                  (k + ".values", c.values, cols[k].values)])
                else:
                    cols[k] = c
            ev = torch.cuda.Event()
            ev.record(side)
        hand = streamcheck.HandOff(count[0], ev, pairs) if check else None
        count[0] += 1
        return Table(cols, num_rows=t.num_rows), ev, fresh, hand

    try:
        nxt = issue(next(it))
    except StopIteration:
        return
    while nxt is not None:
        cur, ev, fresh, hand = nxt
        if ev is not None:
            consumer = torch.cuda.current_stream(dev)
            consumer.wait_event(ev)
            for t in fresh:
                t.record_stream(consumer)
        try:
            nxt = issue(next(it))
        except StopIteration:
            nxt = None
        yield cur
        if hand is not None:  # the consumer queued its work on `cur` and asks for the next batch
            hand.verify(consumer)


def _rebatch(it: Iterator[Table], global_batch: int) -> Iterator[Table]:
    ctx = get_context()
    b = global_batch // ctx.world_size + (1 if global_batch % ctx.world_size > ctx.rank else 0)
    pending: List[Table] = []
    have = 0
    for t in it:
        pending.append(t)
        have += t.num_rows
        while have >= b:
            full = Table.concat(pending) if len(pending) > 1 else pending[0]
            yield full.slice(0, b)
            rest = full.slice(b, full.num_rows)
            pending = [rest] if rest.num_rows else []
            have = rest.num_rows
