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
                   "state": {k: (v.detach().cpu() if isinstance(v, torch.Tensor) else v) for k, v in state.items()}}
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
        # our own files (written by save above); they hold python scalars/lists besides tensors
        payload = torch.load(os.path.join(d, "rank-%d.pt" % ctx.rank), weights_only=False)
        return int(payload["epoch"]), payload["state"]


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
