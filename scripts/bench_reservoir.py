#!/usr/bin/env python3
"""Device reservoir sampler (ops/datagen.py) vs the sequential host sampler: time and equality."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flink_ml_amd.models.kmeans import reservoir_sample_indices  # noqa: E402
from flink_ml_amd.ops.datagen import reservoir_sample_device  # noqa: E402

for n in (12_500_000, 100_000_000):
    reservoir_sample_device(n, 1024, 1, "cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d = reservoir_sample_device(n, 1024, 1, "cuda").cpu().numpy()
    t1 = time.perf_counter()
    h = reservoir_sample_indices(n, 1024, 1)
    t2 = time.perf_counter()
    print(json.dumps({"n": n, "k": 1024, "device_ms": round((t1 - t0) * 1e3, 2), "host_ms": round((t2 - t1) * 1e3, 2),
                      "equal": bool(np.array_equal(d, h))}), flush=True)
