#!/usr/bin/env python3
"""Launch-to-completion latency of a tiny kernel after the GPU sat idle for a while (does the
first launch after idle wait tens of ms?)."""
import time

import torch

dev = torch.device("cuda")
x = torch.zeros(1 << 20, device=dev)
big = torch.randn(4096, 4096, device=dev)
torch.cuda.synchronize()
for idle_ms in (0, 1, 2, 5, 10, 20, 50, 100, 300, 1000):
    res = []
    for _ in range(3):
        big @ big
        torch.cuda.synchronize()
        time.sleep(idle_ms / 1e3)
        t0 = time.perf_counter()
        x.fill_(1.0)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) * 1e3)
    print("idle %5d ms -> tiny kernel + sync %s ms" % (idle_ms, " ".join("%.3f" % r for r in res)), flush=True)
# after a D2H read (as the warm fit's coefficient read-back)
for idle_ms in (0, 2, 30):
    res = []
    for _ in range(3):
        big @ big
        _ = x[:4].cpu()
        time.sleep(idle_ms / 1e3)
        t0 = time.perf_counter()
        x.fill_(1.0)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) * 1e3)
    print("after D2H, idle %3d ms -> %s ms" % (idle_ms, " ".join("%.3f" % r for r in res)), flush=True)
