"""Tracing / metrics (SURVEY §5 "Tracing / profiling", "Metrics / logging").

* ``range(name)`` — a roctx range (visible in ``rocprofv3 --marker-trace`` / ``-r``) plus an
  optional wall-clock record; no-op cost when tracing is off.
* ``MetricGroup`` / ``gauge`` — a tiny metrics registry used for the ``modelDataVersion`` gauge of
  the online models (``OnlineKMeansModel.java:58,163-166``, ``OnlineLogisticRegressionModel.java:59,129-133``)
  that the streaming tests synchronise on.
* ``log_round`` — structured JSON per-round log lines (rank, epoch, loss, weight, ms).
* ``torch_profile(path)`` — a ``torch.profiler`` session (host ops + HIP kernels) exported as a
  Chrome trace per rank (``FMLX_TORCH_PROFILE=<dir>`` or ``bench.py --torch-profile <dir>``).
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import sys
import threading
import time
from typing import Callable, Dict, Optional

_ROCTX = None
_ROCTX_TRIED = False
_ENABLED = os.environ.get("FMLX_TRACE", "0") == "1"
_RECORDS = []


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if _ROCTX_TRIED:
        return _ROCTX
    _ROCTX_TRIED = True
    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _ROCTX = lib
            break
        except OSError:
            continue
    return _ROCTX


def enable(on: bool = True) -> None:
    global _ENABLED
    _ENABLED = on


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    if not _ENABLED:
        yield
        return
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()
        _RECORDS.append((name, (time.perf_counter() - t0) * 1e3))


def records():
    return list(_RECORDS)


_LOG_ROUNDS = os.environ.get("FMLX_LOG_ROUNDS", "0") == "1"
_LOG_SINK = None  # file-like; default stderr


def rounds_enabled() -> bool:
    """Per-round structured logging is on (``FMLX_LOG_ROUNDS=1`` or ``log_rounds(True)``); callers
    only then pay the device syncs / event timings a round record needs."""
    return _LOG_ROUNDS


def log_rounds(on: bool = True, sink=None) -> None:
    global _LOG_ROUNDS, _LOG_SINK
    _LOG_ROUNDS, _LOG_SINK = on, sink


def log_round(**fields) -> None:
    """One JSON line per round: rank, epoch, loss, Σweight, kernel / collective ms, bytes, ..."""
    if _LOG_ROUNDS:
        (_LOG_SINK or sys.stderr).write(json.dumps(fields) + "\n")


def enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def torch_profile(path: Optional[str]):
    """Records a torch.profiler trace of the enclosed work into ``<path>/trace_rank<r>.json``
    (no-op when ``path`` is falsy)."""
    if not path:
        yield None
        return
    import torch
    from torch.profiler import ProfilerActivity, profile

    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    rank = int(os.environ.get("RANK", "0"))
    os.makedirs(path, exist_ok=True)
    with profile(activities=acts, record_shapes=False) as prof:
        yield prof
    prof.export_chrome_trace(os.path.join(path, "trace_rank%d.json" % rank))


class MetricGroup:
    _GLOBAL: Dict[str, Dict[str, Callable]] = {}
    _LOCK = threading.Lock()

    def __init__(self, scope: str):
        self.scope = scope

    def gauge(self, name: str, fn: Callable):
        with MetricGroup._LOCK:
            MetricGroup._GLOBAL.setdefault(self.scope, {})[name] = fn
        return fn

    @staticmethod
    def read(scope: str, name: str):
        fn = MetricGroup._GLOBAL.get(scope, {}).get(name)
        return None if fn is None else fn()

    @staticmethod
    def find(name: str):
        out = {}
        for scope, gauges in MetricGroup._GLOBAL.items():
            if name in gauges:
                out[scope] = gauges[name]()
        return out
