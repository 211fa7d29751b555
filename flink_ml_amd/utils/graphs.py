"""hipGraph capture helper.

``torch.cuda.graph(g)`` synchronises the device and calls ``torch.cuda.empty_cache()`` before
every capture: every cached allocator block goes back to the driver, so the allocations that
follow (the next fit's scratch, the graph's own pool) pay ``hipMalloc`` again — measured 18 ms of
a 61 ms KMeans fit (12.5M × 128, k = 1024, 10 iterations; profiles/r3). ``capture`` records the
same graph on a side stream without emptying the cache and without a device-wide sync.
"""
from __future__ import annotations

from typing import Callable

import torch


_STREAMS = {}


def _capture_stream(device) -> torch.cuda.Stream:
    """One capture stream per device, reused: creating a HIP stream costs ~7 ms on the host
    (hipStreamCreateWithPriority in profiles/r4 sys-traces), once per captured graph before."""
    key = torch.device(device if device is not None else "cuda").index
    if key is None:
        key = torch.cuda.current_device()
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.Stream(key)
    return st


def aux_stream(device, name: str, priority: int = 0) -> torch.cuda.Stream:
    """A named helper stream per (device, name, priority), created once and reused (a fresh
    stream per trainer cost ~7 ms of host time per fit)."""
    idx = torch.device(device).index
    if idx is None:
        idx = torch.cuda.current_device()
    key = (idx, name, priority)
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.Stream(idx, priority=priority)
    return st


def capture(fn: Callable[[], object], device=None) -> torch.cuda.CUDAGraph:
    """Captures the kernels ``fn()`` launches on the current stream into a new CUDAGraph (the
    launches are recorded, not executed) and returns it; stream-ordered after the work already
    queued on the current stream."""
    g = torch.cuda.CUDAGraph()
    cur = torch.cuda.current_stream(device)
    side = _capture_stream(device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        g.capture_begin()
        try:
            fn()
        finally:
            g.capture_end()
    cur.wait_stream(side)
    return g
