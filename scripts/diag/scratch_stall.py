#!/usr/bin/env python3
"""Does the first launch after a scratch-using kernel (hipCUB onesweep: 80 B private segment)
stall the queue? Latency of a tiny fill + sync after: a scratch kernel, a plain kernel, with
idle gaps. Env knobs under test: HSA_NO_SCRATCH_RECLAIM, HSA_ENABLE_SCRATCH_ASYNC_RECLAIM."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flink_ml_amd.ops import native  # noqa: E402

dev = torch.device("cuda")
m = 8 << 20
key = torch.randint(0, 1 << 20, (m,), dtype=torch.int32, device=dev)
iota = torch.arange(m, dtype=torch.int32, device=dev)
ko, vo = torch.empty_like(key), torch.empty_like(key)
lib = native.kernels()
tb = int(lib.fmlx_sort_pairs_temp_bytes(m, 20))
temp = torch.empty(tb, dtype=torch.uint8, device=dev)
x = torch.zeros(1 << 20, device=dev)


def scratch_kernel():
    native.call("fmlx_sort_pairs", native.ptr(key), native.ptr(ko), native.ptr(iota), native.ptr(vo), m, 20,
                native.ptr(temp), tb, native.stream_ptr(dev))


def plain_kernel():
    torch.add(key, 1, out=ko)


print({k: os.environ.get(k) for k in ("HSA_NO_SCRATCH_RECLAIM", "HSA_ENABLE_SCRATCH_ASYNC_RECLAIM")}, flush=True)
for name, fn in (("plain", plain_kernel), ("scratch", scratch_kernel)):
    for idle_ms in (0, 2, 10, 50):
        res = []
        for _ in range(4):
            fn()
            torch.cuda.synchronize()
            time.sleep(idle_ms / 1e3)
            t0 = time.perf_counter()
            x.fill_(1.0)
            torch.cuda.synchronize()
            res.append((time.perf_counter() - t0) * 1e3)
        print("%-8s then idle %3d ms -> fill+sync %s ms" % (name, idle_ms, " ".join("%.3f" % r for r in res)),
              flush=True)
# the trainer's pattern: scratch kernel, read back (D2H), host work, new launches
res = []
for _ in range(4):
    scratch_kernel()
    _ = vo[:1].item()
    time.sleep(0.002)
    t0 = time.perf_counter()
    x.fill_(2.0)
    _ = x[:1].item()
    res.append((time.perf_counter() - t0) * 1e3)
print("scratch, item, 2 ms host, fill + item: %s ms" % " ".join("%.3f" % r for r in res), flush=True)
