#!/usr/bin/env python3
"""Why a 4 MB torch.zeros on the device can cost ~25 ms: allocator stats around fresh allocations
after large frees (the SVC whole fit's coefficient vector)."""
import time

import torch

dev = torch.device("cuda")
keys = ("num_alloc_retries", "segment.all.allocated", "segment.all.freed", "num_device_alloc", "num_device_free")


def stats():
    s = torch.cuda.memory_stats(dev)
    return {k: s.get(k, 0) for k in keys}


def tm(label, fn):
    torch.cuda.synchronize()
    a = stats()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    b = stats()
    print("%-46s %8.3f ms  %s" % (label, ms, {k: b[k] - a[k] for k in keys if b[k] != a[k]}), flush=True)
    return out


big = tm("alloc 3.2 GB (empty)", lambda: torch.empty(800_000_000, dtype=torch.float32, device=dev))
tm("zeros 4 MB", lambda: torch.zeros(1 << 20, device=dev))
tm("zeros 4 MB again", lambda: torch.zeros(1 << 20, device=dev))
keep = [tm("zeros 4 MB kept #%d" % i, lambda: torch.zeros(1 << 20, device=dev)) for i in range(6)]
tm("zeros 64 MB", lambda: torch.zeros(16 << 20, device=dev))
tm("zeros 256 MB", lambda: torch.zeros(64 << 20, device=dev))
tm("zeros 1 GB", lambda: torch.zeros(256 << 20, device=dev))
del big
tm("zeros 4 MB after freeing 3.2 GB", lambda: torch.zeros(1 << 20, device=dev))
tm("raw hipMalloc path: empty 20 MB", lambda: torch.empty(5 << 20, device=dev))
