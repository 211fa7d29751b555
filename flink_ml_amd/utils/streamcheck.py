"""Stream-ordering checks for cross-stream hand-offs (SURVEY §5 "race detection").

The reference relies on Flink's single-threaded mailbox per task, so it has no data races by
construction. Here the one place where device data crosses HIP streams is the ingestion path:
``stream._prefetch`` copies batch k+1 host→HBM on a side stream while the consumer stream runs
batch k, and hands the copies over with ``wait_event`` + ``record_stream``. A missing wait, or
an allocator block reused while a consumer kernel still reads it (the class of bug
``record_stream`` prevents), shows up as a batch whose device bytes differ from its source.

``FMLX_STREAM_CHECK=1`` turns on a checker for every hand-off: when the batch is handed out,
an order-independent checksum of every host source column is taken; when the consumer asks for
the next batch (its work on this one is queued), the consumer stream is synchronised, the
producing event must have completed, and the device copy's checksum must equal the source's.
Any violation raises ``StreamOrderError`` naming the batch and column. Slow (host checksums,
one sync per batch) and off by default, like ``FMLX_SYNC_CHECK`` for kernel faults.
"""
from __future__ import annotations

import os
from typing import List, Tuple

import torch


class StreamOrderError(RuntimeError):
    """A cross-stream hand-off observed data that does not match what the producer wrote."""


def enabled() -> bool:
    return os.environ.get("FMLX_STREAM_CHECK", "0") == "1"


def checksum(t: torch.Tensor) -> Tuple[int, int]:
    """(Σ bytes, Σ byte·position mod 2^31) over the raw bytes: order-sensitive enough to catch
    swapped or partially written chunks, identical on host and device."""
    b = t.detach().contiguous().view(-1).view(torch.uint8).to(torch.int64)
    if b.numel() == 0:
        return 0, 0
    pos = torch.arange(b.numel(), device=b.device, dtype=torch.int64) % 65521 + 1
    return int(b.sum()), int((b * pos).sum() % (1 << 31))


class HandOff:
    """One batch handed from the producing stream to the consumer stream."""

    def __init__(self, index: int, event: "torch.cuda.Event", pairs: List[Tuple[str, torch.Tensor, torch.Tensor]]):
        # pairs: (column name, host source, device copy)
        self.index = index
        self.event = event
        self.pairs = [(name, dev, checksum(src)) for name, src, dev in pairs]

    def verify(self, consumer: "torch.cuda.Stream") -> None:
        consumer.synchronize()
        if not self.event.query():
            raise StreamOrderError("batch %d: the consumer stream finished its work while the H2D copy it "
                                   "was handed had not completed (missing wait_event)" % self.index)
        for name, dev, want in self.pairs:
            got = checksum(dev)
            if got != want:
                raise StreamOrderError("batch %d, column %r: device copy %s differs from its host source %s "
                                       "(stream-ordering race on the hand-off)" % (self.index, name, got, want))
