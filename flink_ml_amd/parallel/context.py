"""SPMD execution context: one process per GPU.

Replaces Flink's JobManager/TaskManager/subtask model: every rank runs the
same driver program over its own data partition, in lockstep; there is no dataflow graph and
no coordinator. Rank/world come from ``torch.distributed`` (env:// rendezvous — RANK,
WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT, as set by ``torch.distributed.run``). The
collective backend is ``nccl`` (= RCCL on ROCm, over xGMI) when GPUs are present and ``gloo``
on CPU-only hosts (tests).
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class SPMDContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None
    forced: bool = False  # FMLX_FORCE_PG=1: a process group (and its collectives) even at world 1
    sharers: int = 1  # ranks of the group on this rank's physical GPU (measured at init, see below)

    @property
    def is_distributed(self) -> bool:
        return (self.world_size > 1 or self.forced) and dist.is_available() and dist.is_initialized()

    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    def barrier(self) -> None:
        if self.is_distributed:
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index or 0])
            else:
                dist.barrier()


_CTX: Optional[SPMDContext] = None
_LOCK = threading.Lock()


def _gpu_available() -> bool:
    if os.environ.get("FMLX_DEVICE", "").lower() == "cpu":
        return False
    try:
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def default_device(local_rank: int = 0) -> torch.device:
    forced = os.environ.get("FMLX_DEVICE")
    if forced and forced.lower() != "cpu" and forced.lower() != "cuda":
        return torch.device(forced)
    if _gpu_available():
        n = torch.cuda.device_count()
        return torch.device("cuda", local_rank % max(n, 1))
    return torch.device("cpu")


def _rendezvous_store(world: int, forced: bool, timeout_s: int):
    """The store the process group rendezvous on, or None for torch's env:// default.

    - FMLX_FORCE_PG at world 1: an in-process ``HashStore``; no socket is bound at all.
    - ``FMLX_STORE=host:port``: a TCPStore some parent already hosts (``tests/spmd.py`` binds it
      with port 0 and hands out the port it got); every rank connects as a client. This never
      binds-then-closes a port, so two concurrent groups cannot race for the same number.
    """
    import datetime

    if forced:
        return dist.HashStore()
    spec = os.environ.get("FMLX_STORE")
    if spec:
        host, port = spec.rsplit(":", 1)
        return dist.TCPStore(host, int(port), world, is_master=False,
                             timeout=datetime.timedelta(seconds=timeout_s))
    return None


def force_pg() -> bool:
    """FMLX_FORCE_PG=1: create the process group even at WORLD_SIZE=1, so every collective of the
    distributed code path (RCCL all-reduces, hipGraph-captured ones included; the xGMI set-up and
    its fallback) runs on a one-GPU host exactly as it would on eight."""
    return os.environ.get("FMLX_FORCE_PG", "0") == "1"


def init_distributed(backend: Optional[str] = None, timeout_s: int = 600) -> SPMDContext:
    """Initialises the process group from the environment (idempotent)."""
    global _CTX
    with _LOCK:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
        device = default_device(local_rank)
        if device.type == "cuda":
            torch.cuda.set_device(device)
        forced = world == 1 and force_pg()
        if (world > 1 or forced) and not dist.is_initialized():
            import datetime

            if backend is None:
                # FMLX_BACKEND=gloo: several ranks sharing one GPU (rehearsals of multi-GPU paths)
                backend = os.environ.get("FMLX_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kwargs = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
            store = _rendezvous_store(world, forced, timeout_s)
            if store is not None:
                kwargs.update(store=store, rank=rank, world_size=world)
            if backend == "nccl":
                kwargs["device_id"] = device
            dist.init_process_group(**kwargs)
        if dist.is_initialized():
            backend = dist.get_backend()
            world = dist.get_world_size()
            rank = dist.get_rank()
            forced = world == 1
        _CTX = SPMDContext(rank=rank, world_size=world, local_rank=local_rank, device=device, backend=backend,
                           forced=forced)
        if _CTX.is_distributed and _CTX.is_gpu and world > 1:
            _CTX.sharers = _measure_sharers(_CTX)
    if _CTX.is_gpu:
        from . import xgmi  # noqa: F401  (imported here, at set-up, not inside the first fit)

        if _CTX.is_distributed and backend == "nccl":
            xgmi.get()  # collective set-up of the one-shot xGMI exchange, at a point every rank reaches
    return _CTX


def device_identity(device: torch.device) -> str:
    """Host name + PCI domain:bus:device of ``device``: equal strings = the same physical GPU,
    whatever HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES renumbering each process sees."""
    import socket

    p = torch.cuda.get_device_properties(device)
    return "%s/%04x:%02x:%02x" % (socket.gethostname(), p.pci_domain_id, p.pci_bus_id, p.pci_device_id)


def count_sharers(ids, rank: int) -> int:
    """Ranks whose device identity equals ``rank``'s (itself included)."""
    return sum(1 for i in ids if i == ids[rank])


def _measure_sharers(ctx: SPMDContext) -> int:
    """All-gathers every rank's device identity once at init (one tiny collective every rank
    reaches) and counts the ranks on this rank's GPU: 1 with a GPU per rank; every rank in the
    one-GPU multi-rank rehearsals (``FMLX_DEVICE=cuda:0`` for all ranks)."""
    ids = [None] * ctx.world_size
    dist.all_gather_object(ids, device_identity(ctx.device))
    return count_sharers(ids, ctx.rank)


def device_sharers(ctx: SPMDContext) -> int:
    """Ranks of the group running on this rank's physical GPU (measured at ``init_distributed``
    by comparing PCI ids, so per-process visible-device masks cannot fool it)."""
    if not ctx.is_gpu or ctx.world_size <= 1:
        return 1
    return max(1, int(ctx.sharers))


def get_context() -> SPMDContext:
    global _CTX
    if _CTX is None:
        if dist.is_available() and dist.is_initialized():
            return init_distributed()
        with _LOCK:
            if _CTX is None:
                _CTX = SPMDContext(device=default_device(0))
    return _CTX


def set_context(ctx: SPMDContext) -> None:
    global _CTX
    _CTX = ctx


def reset_context() -> None:
    global _CTX
    _CTX = None


def shutdown() -> None:
    global _CTX
    from . import xgmi

    xgmi.reset()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _CTX = None
