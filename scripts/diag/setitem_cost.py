#!/usr/bin/env python3
"""Host cost of `cuda_tensor[i] = python_scalar` vs an explicit fill_, idle and behind queued work."""
import time

import torch

dev = torch.device("cuda")
t = torch.zeros(8, dtype=torch.int32, device=dev)
f = torch.zeros(1 << 20, dtype=torch.float32, device=dev)
big = torch.randn(8192, 8192, device=dev)
torch.cuda.synchronize()


def tm(label, fn, busy=False, reps=5):
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        if busy:
            for _ in range(4):
                big @ big  # ~ms of queued work
        t0 = time.perf_counter()
        fn()
        out.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    print("%-40s %s ms" % (label, " ".join("%.3f" % x for x in out)), flush=True)


tm("int32 t[1] = 1 (idle)", lambda: t.__setitem__(1, 1))
tm("int32 t[1:2].fill_(1) (idle)", lambda: t[1:2].fill_(1))
tm("f32 f[5] = 2.5 (idle)", lambda: f.__setitem__(5, 2.5))
tm("int32 t[1] = 1 (busy)", lambda: t.__setitem__(1, 1), busy=True)
tm("int32 t[1:2].fill_(1) (busy)", lambda: t[1:2].fill_(1), busy=True)
tm("f32 f[5] = 2.5 (busy)", lambda: f.__setitem__(5, 2.5), busy=True)
tm("torch.zeros(8, cuda) (busy)", lambda: torch.zeros(8, dtype=torch.int32, device=dev), busy=True)
tm("torch.tensor([..], cuda) (busy)", lambda: torch.tensor([0, 1, 0, 0], dtype=torch.int32, device=dev), busy=True)
