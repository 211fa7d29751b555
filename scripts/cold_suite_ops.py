#!/usr/bin/env python3
"""Which torch ops still pay a first-use cost in the cold reference suite: runs every config of
bench/conf/reference-suite.json once (after the CLI's warm_runtime) under a dispatch mode that
times each aten op with a device sync around it, and prints one JSON line per config with its
total time and the ops slower than ``--min-ms`` (default 10 ms) — in a fresh process those are
torch's lazy code-object loads, the part of the cold suite the library's own kernels do not set.
Usage: python scripts/cold_suite_ops.py [--pattern REGEX] [--max-values N]
"""
import argparse
import json
import os
import re
import sys
import time
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class OpTimer(TorchDispatchMode):
    def __init__(self, min_ms):
        super().__init__()
        self.min_ms = min_ms
        self.slow = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        if torch.cuda.is_current_stream_capturing():  # (inside a hipGraph capture: no sync)
            return func(*args, **(kwargs or {}))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = func(*args, **(kwargs or {}))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        if dt >= self.min_ms:  # with the innermost library frame that called it
            site = ""
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "flink_ml_amd" in fr.filename:
                    site = "%s:%d" % (fr.filename.split("flink_ml_amd/")[-1], fr.lineno)
                    break
            self.slow.append((str(func), round(dt, 1), site))
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pattern", default=None)
    ap.add_argument("--max-values", type=int, default=1_000_000)
    ap.add_argument("--min-ms", type=float, default=10.0)
    ap.add_argument("--warm", action="store_true", help="run each config once first (warm op profile)")
    a = ap.parse_args()
    from flink_ml_amd.bench import runner

    runner.warm_runtime()
    conf = runner.load_config("flink_ml_amd/bench/conf/reference-suite.json")
    rx = re.compile(a.pattern) if a.pattern else None
    for name, spec in conf.items():
        if name == "version" or (rx and not rx.match(name)):
            continue
        spec = runner._cap_values(spec, a.max_values)
        if a.warm:
            runner.run_benchmark(name, spec)
        m = OpTimer(a.min_ms)
        t0 = time.perf_counter()
        try:
            with m:
                runner.run_benchmark(name, spec)
            err = None
        except Exception as e:  # noqa: BLE001
            err = "%s: %s" % (type(e).__name__, e)
        print(json.dumps({"config": name, "ms": round((time.perf_counter() - t0) * 1e3, 1), "slow_ops": m.slow,
                          "error": err}), flush=True)


if __name__ == "__main__":
    main()
