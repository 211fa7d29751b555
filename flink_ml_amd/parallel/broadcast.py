"""Broadcast variables (reference ``CORE/common/broadcast/BroadcastUtils.java:64-191``,
``BroadcastContext.java:34-113``, ``operator/BroadcastVariableReceiverOperator.java:45-155``,
``operator/AbstractBroadcastWrapperOperator.java:283-374``).

Reference semantics: ``withBroadcastStream(inputs, {name: stream}, func)`` delivers EVERY record
of each broadcast stream to every subtask (``stream.broadcast()``), caches them in a JVM-static
``BroadcastContext`` keyed ``name-subtaskIdx``, buffers the non-broadcast inputs until all
broadcast inputs have finished, then runs ``func`` whose operators read the records through
``getBroadcastVariable(name)``.

SPMD equivalent: a broadcast variable is materialised once per rank before ``fn`` runs — the
union of all ranks' records (an all-gather; RCCL for device tensors) unless the value is already
replicated (``Table.replicated``, or ``replicated=True``, e.g. model data every rank holds).
There is nothing to buffer: inputs are resident partitions and ``fn`` simply runs after the
gather. The registry is process-local (the JVM-static map's analogue) and is cleared when the
call returns, like the reference's ``BroadcastContext.remove`` at operator close.
"""
from __future__ import annotations

import threading
from typing import Any, Callable, Dict, Sequence

import torch

from ..table import Table
from . import comm
from .context import get_context

_LOCK = threading.Lock()
_REGISTRY: Dict[str, Any] = {}


class BroadcastContext:
    """Process-local store of materialised broadcast variables (``BroadcastContext.java``)."""

    @staticmethod
    def put(key: str, value: Any) -> None:
        with _LOCK:
            _REGISTRY[key] = value

    @staticmethod
    def get(key: str) -> Any:
        with _LOCK:
            if key not in _REGISTRY:
                raise KeyError("broadcast variable %s is not available" % key)
            return _REGISTRY[key]

    @staticmethod
    def remove(key: str) -> None:
        with _LOCK:
            _REGISTRY.pop(key, None)


class BroadcastRuntimeContext:
    """What ``fn`` receives: ``get_broadcast_variable(name)`` (``BroadcastStreamingRuntimeContext.java:71``)."""

    def __init__(self, keys: Dict[str, str]):
        self._keys = keys

    def get_broadcast_variable(self, name: str) -> Any:
        if name not in self._keys:
            raise KeyError("no broadcast variable named %s" % name)
        return BroadcastContext.get(self._keys[name])

    getBroadcastVariable = get_broadcast_variable


def _materialise(value: Any, replicated: bool) -> Any:
    if replicated or not get_context().is_distributed:
        return value
    if isinstance(value, Table):
        if value.replicated:
            return value
        parts = comm.all_gather_object(value.to("cpu"))
        full = Table.concat([p for p in parts if p is not None and p.num_rows]) if parts else value
        return full.as_replicated()
    if isinstance(value, torch.Tensor):
        return comm.all_gather_cat(value)
    return [x for part in comm.all_gather_object(list(value)) for x in part]


def with_broadcast_stream(inputs: Sequence[Any], broadcast: Dict[str, Any],
                          fn: Callable[[Sequence[Any], BroadcastRuntimeContext], Any],
                          replicated: bool = False) -> Any:
    """Runs ``fn(inputs, ctx)`` with every entry of ``broadcast`` available on every rank as
    ``ctx.get_broadcast_variable(name)``. ``replicated=True`` declares the values identical on
    every rank already (no gather)."""
    rank = get_context().rank
    keys = {}
    try:
        for name, value in broadcast.items():
            key = "%s-%d" % (name, rank)
            BroadcastContext.put(key, _materialise(value, replicated))
            keys[name] = key
        return fn(inputs, BroadcastRuntimeContext(keys))
    finally:
        for key in keys.values():
            BroadcastContext.remove(key)
