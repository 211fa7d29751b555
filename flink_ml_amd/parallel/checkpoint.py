"""Round-level checkpoint / resume and fault injection (SURVEY §5 "Failure detection / elastic
recovery / fault injection", "Checkpoint / resume").

The reference relies on Flink's aligned checkpoints: operator ``ListState`` (SGD keeps coefficient,
feedback array, ``nextBatchOffset``; ``SGD.java:307-363``), the iteration head logs feedback
records between barriers (``HeadOperator.java:98-116``), and recovery with a different
parallelism is rejected (``HeadOperator.java:197-208``). In the SPMD engine the equivalent is a
consistent round checkpoint:

* every rank writes its algorithm state for round ``e`` (``round-<e>/<name>-rank<r>.pt``), the ranks
  barrier, and rank 0 atomically publishes ``_COMMITTED`` — a half-written round is never restored;
* ``restore(name)`` loads the newest committed round; the world size must match (no rescaling,
  like the reference);
* failures surface as exceptions (a dead peer makes RCCL/gloo collectives raise; the process-group
  timeout is the watchdog); the launcher (``torchrun --max-restarts``) restarts every rank and the
  algorithms resume from the checkpoint. ``TORCHELASTIC_RESTART_COUNT`` / ``FMLX_ATTEMPT`` give the
  attempt number;
* ``FailAfter`` mirrors the reference's ``FailingMap`` test operator: it throws once, on one rank,
  in one attempt, after a given number of rounds.

Checkpointing is switched on per process with ``enable(path, interval)`` (or the env vars
``FMLX_CHECKPOINT_DIR`` / ``FMLX_CHECKPOINT_INTERVAL``); each algorithm invocation gets a
deterministic name (call counter + algorithm) so a restarted job finds its own state.
"""
from __future__ import annotations

import os
import re
import shutil
from typing import Any, Dict, List, Optional, Tuple

import torch

from .context import get_context

_PKG = __name__.split(".")[0] + "."


def _encode(v):
    """Checkpoint payload → tensors, python scalars/strings and containers only, so restore can
    use the weights-only unpickler. numpy arrays/scalars become tagged tensors; objects of this
    package's own classes (DenseVector, …) become tagged attribute dicts."""
    import numpy as np

    if isinstance(v, torch.Tensor):
        return v.detach().cpu()
    if isinstance(v, np.generic):  # before the python types: np.float64 is a float subclass
        return v.item()
    if v is None or isinstance(v, (bool, int, float, str, bytes)):
        return v
    if isinstance(v, np.ndarray):
        if v.dtype != object:
            try:
                return {"__np__": torch.from_numpy(np.ascontiguousarray(v))}
            except TypeError:  # strings, bytes, datetimes, unsigned widths torch cannot hold
                if v.dtype.kind in "Mm":  # datetime64 / timedelta64: their int64 ticks
                    return {"__npt__": v.dtype.str, "shape": list(v.shape),
                            "ticks": torch.from_numpy(np.ascontiguousarray(v).view(np.int64).reshape(-1))}
                return {"__npt__": v.dtype.str, "shape": list(v.shape), "data": _encode(v.reshape(-1).tolist())}
        return {"__np__": _encode(v.tolist())}
    if isinstance(v, dict):
        return {"__dict__": [[_encode(k), _encode(x)] for k, x in v.items()]}
    if isinstance(v, tuple):
        return {"__tuple__": [_encode(x) for x in v]}
    if isinstance(v, list):
        return [_encode(x) for x in v]
    cls = type(v)
    if cls.__module__.startswith(_PKG):
        attrs = dict(vars(v)) if hasattr(v, "__dict__") else {}
        for klass in cls.__mro__:
            for a in getattr(klass, "__slots__", ()):
                if a != "__dict__" and hasattr(v, a):
                    attrs[a] = getattr(v, a)
        return {"__obj__": "%s:%s" % (cls.__module__, cls.__qualname__), "attrs": _encode(attrs)}
    raise TypeError("checkpoint state of type %s.%s cannot be saved (tensors, numpy arrays, python scalars, "
                    "containers and %s* objects only)" % (cls.__module__, cls.__qualname__, _PKG))


def _decode(v):
    import importlib

    if isinstance(v, list):
        return [_decode(x) for x in v]
    if not isinstance(v, dict):
        return v
    if "__np__" in v:
        x = v["__np__"]
        return x.numpy() if isinstance(x, torch.Tensor) else __import__("numpy").array(_decode(x), dtype=object)
    if "__npt__" in v:
        import numpy as np

        dt = np.dtype(v["__npt__"])
        if "ticks" in v:
            return v["ticks"].numpy().view(dt).reshape(v["shape"])
        return np.array(_decode(v["data"]), dtype=dt).reshape(v["shape"])
    if "__tuple__" in v:
        return tuple(_decode(x) for x in v["__tuple__"])
    if "__dict__" in v:
        return {_decode(k): _decode(x) for k, x in v["__dict__"]}
    if "__obj__" in v:
        mod, name = v["__obj__"].split(":")
        if not mod.startswith(_PKG):  # only this package's classes are ever rebuilt
            raise ValueError("checkpoint names a foreign class %s" % v["__obj__"])
        cls = importlib.import_module(mod)
        for part in name.split("."):
            cls = getattr(cls, part)
        obj = object.__new__(cls)
        for a, x in _decode(v["attrs"]).items():
            object.__setattr__(obj, a, x)
        return obj
    return {k: _decode(x) for k, x in v.items()}


class InjectedFailure(RuntimeError):
    """Raised by ``FailAfter`` (the analogue of the reference's FailingMap exception)."""


def attempt() -> int:
    for k in ("FMLX_ATTEMPT", "TORCHELASTIC_RESTART_COUNT"):
        if k in os.environ:
            return int(os.environ[k])
    return 0


class FailAfter:
    """Throws ``InjectedFailure`` when round ``rounds`` is reached on ``rank`` in ``on_attempt``."""

    def __init__(self, rounds: int, rank: int = 0, on_attempt: int = 0):
        self.rounds, self.rank, self.on_attempt = int(rounds), int(rank), int(on_attempt)

    def check(self, epoch: int) -> None:
        if epoch == self.rounds and get_context().rank == self.rank and attempt() == self.on_attempt:
            raise InjectedFailure("injected failure at round %d on rank %d (attempt %d)"
                                  % (epoch, self.rank, self.on_attempt))


_FAULTS: List[FailAfter] = []


def inject(fault: FailAfter) -> None:
    _FAULTS.append(fault)


def clear_faults() -> None:
    _FAULTS.clear()


def fault_point(epoch: int) -> None:
    """Called by the iteration drivers at the start of every round."""
    for f in _FAULTS:
        f.check(epoch)


class CheckpointManager:
    def __init__(self, path: str, interval: int = 1, keep: int = 2):
        self.path = path
        self.interval = max(1, int(interval))
        self.keep = max(1, int(keep))
        self._calls = 0
        os.makedirs(path, exist_ok=True)

    def next_name(self, algorithm: str) -> str:
        """Deterministic per-invocation name: the n-th checkpointed call of this process."""
        self._calls += 1
        return "%04d-%s" % (self._calls, algorithm)

    def due(self, epoch: int) -> bool:
        return epoch > 0 and epoch % self.interval == 0

    def _round_dir(self, name: str, epoch: int) -> str:
        return os.path.join(self.path, name, "round-%08d" % epoch)

    def save(self, name: str, epoch: int, state: Dict[str, Any]) -> None:
        from . import comm

        ctx = get_context()
        d = self._round_dir(name, epoch)
        os.makedirs(d, exist_ok=True)
        payload = {"epoch": epoch, "world_size": ctx.world_size, "rank": ctx.rank,
                   "state": _encode(dict(state))}
        tmp = os.path.join(d, ".rank-%d.tmp" % ctx.rank)
        torch.save(payload, tmp)
        os.replace(tmp, os.path.join(d, "rank-%d.pt" % ctx.rank))
        comm.barrier()
        if ctx.rank == 0:
            mk = os.path.join(d, ".committed.tmp")
            with open(mk, "w") as f:
                f.write("%d\n" % ctx.world_size)
            os.replace(mk, os.path.join(d, "_COMMITTED"))
            self._gc(name)
        comm.barrier()

    def _rounds(self, name: str) -> List[int]:
        base = os.path.join(self.path, name)
        if not os.path.isdir(base):
            return []
        out = []
        for e in os.listdir(base):
            m = re.match(r"round-(\d+)$", e)
            if m and os.path.exists(os.path.join(base, e, "_COMMITTED")):
                out.append(int(m.group(1)))
        return sorted(out)

    def _gc(self, name: str) -> None:
        for e in self._rounds(name)[:-self.keep]:
            shutil.rmtree(self._round_dir(name, e), ignore_errors=True)

    def restore(self, name: str) -> Optional[Tuple[int, Dict[str, Any]]]:
        ctx = get_context()
        rounds = self._rounds(name)
        if not rounds:
            return None
        d = self._round_dir(name, rounds[-1])
        with open(os.path.join(d, "_COMMITTED")) as f:
            ws = int(f.read().strip() or 0)
        if ws != ctx.world_size:
            raise RuntimeError("Checkpoint %s was written by %d ranks; recovery with %d ranks is not supported "
                               "(no rescaling, like the reference)." % (d, ws, ctx.world_size))
        # tensors, python scalars, strings, lists and dicts only: the weights-only unpickler
        # executes nothing from a (possibly shared) checkpoint directory
        payload = torch.load(os.path.join(d, "rank-%d.pt" % ctx.rank), weights_only=True)
        return int(payload["epoch"]), _decode(payload["state"])


_ACTIVE: Optional[CheckpointManager] = None


def enable(path: str, interval: int = 1, keep: int = 2) -> CheckpointManager:
    global _ACTIVE
    _ACTIVE = CheckpointManager(path, interval, keep)
    return _ACTIVE


def disable() -> None:
    global _ACTIVE
    _ACTIVE = None


def active() -> Optional[CheckpointManager]:
    global _ACTIVE
    if _ACTIVE is None and os.environ.get("FMLX_CHECKPOINT_DIR"):
        _ACTIVE = CheckpointManager(os.environ["FMLX_CHECKPOINT_DIR"],
                                    int(os.environ.get("FMLX_CHECKPOINT_INTERVAL", "1")))
    return _ACTIVE


class AlgorithmCheckpoint:
    """Per-invocation helper used by the trainers: ``restore()`` once, ``maybe_save(epoch, state)``
    every round, ``fault_point(epoch)`` for injected failures."""

    def __init__(self, algorithm: str):
        self.mgr = active()
        self.name = self.mgr.next_name(algorithm) if self.mgr is not None else None

    def restore(self) -> Optional[Tuple[int, Dict[str, Any]]]:
        return self.mgr.restore(self.name) if self.mgr is not None else None

    def maybe_save(self, epoch: int, state_fn) -> None:
        if self.mgr is not None and self.mgr.due(epoch):
            self.mgr.save(self.name, epoch, state_fn())

    @property
    def interval(self) -> int:
        return self.mgr.interval if self.mgr is not None else 0
