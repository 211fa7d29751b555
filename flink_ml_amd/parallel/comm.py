"""Collectives over RCCL (xGMI) / gloo.

Maps the reference's communication components (SURVEY §2.2 C1–C11, §2.3) onto device-tensor
collectives:

=========================================  ==============================================
reference                                  here
=========================================  ==============================================
``AllReduceImpl.allReduceSum`` (C2)        ``all_reduce_sum``: one-shot xGMI kernel for device
                                           tensors up to 1M elements (``xgmi.py``), else RCCL
gather-to-one ``countWindowAll(P).reduce``  ``all_reduce_sum`` (result replicated, no bcast)
  + broadcast (C3)
``DataStreamUtils.reduce/aggregate`` (C4)  ``all_reduce_*`` for fixed-size accumulators,
                                           ``all_gather_object`` for variable-size ones
broadcast variables (C5)                   ``broadcast_object`` / ``broadcast_tensor``
range / hash shuffles (C10, C11)           ``all_to_all_v``
round alignment (C7)                       implicit SPMD lockstep (+ ``all_reduce`` of flags)
=========================================  ==============================================

All functions are no-ops (or identity) at world size 1, so single-GPU runs pay no
communication. Tensors are moved to the backend's device (``nccl`` → GPU, ``gloo`` → CPU)
and results come back on the caller's device.
"""
from __future__ import annotations

import sys
from typing import Any, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..utils import tracing
from .context import get_context


def _backend_device(ctx):
    return ctx.device if ctx.backend == "nccl" else torch.device("cpu")


def _to_backend(t: torch.Tensor, ctx):
    dev = _backend_device(ctx)
    if t.device != dev:
        return t.to(dev), True
    return t, False


def all_reduce(t: torch.Tensor, op: str = "sum") -> torch.Tensor:
    """In-place all-reduce; returns ``t``. ``op`` in {sum, max, min, prod}."""
    ctx = get_context()
    if not ctx.is_distributed:
        return t
    if tracing.enabled():  # roctx range per collective (name carries op and bytes)
        with tracing.range("allreduce.%s[%dB]" % (op, t.numel() * t.element_size())):
            return _all_reduce(t, op, ctx)
    return _all_reduce(t, op, ctx)


def _all_reduce(t: torch.Tensor, op: str, ctx) -> torch.Tensor:
    if op == "sum" and t.is_cuda:
        x = _xgmi().get()
        if x is not None and x.accepts(t):
            return x.all_reduce_(t)  # one-shot xGMI kernel (small payloads, bit-identical on all ranks)
    rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
           "prod": dist.ReduceOp.PRODUCT}[op]
    work, moved = _to_backend(t, ctx)
    if not work.is_contiguous():
        work = work.contiguous()
        moved = True
    dist.all_reduce(work, op=rop)
    if moved:
        t.copy_(work.to(t.device))
    return t


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    return all_reduce(t, "sum")


def check_collectives() -> None:
    """Raises if an earlier one-shot xGMI collective of this process gave up waiting for a peer
    (its output was poisoned with NaN). No device sync: call it after a host sync point so the
    kernels in question have finished."""
    if "flink_ml_amd.parallel.xgmi" not in sys.modules:
        return  # no xGMI collective has run in this process (a 1-GPU fit never imports it)
    _xgmi().check()


def _xgmi():
    # imported on first use (parallel/xgmi.py imports this package's context); the module import
    # itself is cheap, but a first import inside a fit was a few ms of its wall time
    from . import xgmi

    return xgmi


def all_reduce_scalar(x: float, op: str = "sum", dtype=torch.float64) -> float:
    ctx = get_context()
    if not ctx.is_distributed:
        return x
    t = torch.tensor([x], dtype=dtype, device=_backend_device(ctx))
    all_reduce(t, op)
    v = t.item()  # host sync: every earlier collective on this stream has finished
    check_collectives()
    return v


def all_agree(flag: bool) -> bool:
    """True iff ``flag`` holds on every rank: one MIN over the process group itself (never the
    xGMI exchange, and no check of it), so ranks can agree on leaving a failed exchange."""
    ctx = get_context()
    if not ctx.is_distributed:
        return bool(flag)
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=_backend_device(ctx))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def broadcast_tensor(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    ctx = get_context()
    if not ctx.is_distributed:
        return t
    work, moved = _to_backend(t.contiguous(), ctx)
    dist.broadcast(work, src=src)
    if moved or work.data_ptr() != t.data_ptr():
        t.copy_(work.to(t.device))
    return t


def broadcast_object(obj: Any, src: int = 0) -> Any:
    ctx = get_context()
    if not ctx.is_distributed:
        return obj
    lst = [obj if ctx.rank == src else None]
    dist.broadcast_object_list(lst, src=src, device=_backend_device(ctx))
    return lst[0]


def all_gather_object(obj: Any) -> List[Any]:
    ctx = get_context()
    if not ctx.is_distributed:
        return [obj]
    out: List[Any] = [None] * ctx.world_size
    dist.all_gather_object(out, obj)
    return out


def all_gather_tensor(t: torch.Tensor) -> List[torch.Tensor]:
    """Gathers tensors that may differ in their first dimension."""
    ctx = get_context()
    if not ctx.is_distributed:
        return [t]
    work, _ = _to_backend(t.contiguous(), ctx)
    n = torch.tensor([work.shape[0]], dtype=torch.int64, device=work.device)
    sizes = [torch.zeros_like(n) for _ in range(ctx.world_size)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    pad_shape = (mx,) + tuple(work.shape[1:])
    padded = torch.zeros(pad_shape, dtype=work.dtype, device=work.device)
    padded[: work.shape[0]] = work
    outs = [torch.zeros_like(padded) for _ in range(ctx.world_size)]
    dist.all_gather(outs, padded)
    return [o[:s].to(t.device) for o, s in zip(outs, sizes)]


def all_gather_cat(t: torch.Tensor) -> torch.Tensor:
    return torch.cat(all_gather_tensor(t), dim=0)


def all_to_all_v(chunks: Sequence[torch.Tensor]) -> List[torch.Tensor]:
    """Sends ``chunks[r]`` to rank r; returns the list received from every rank (C10/C11)."""
    ctx = get_context()
    if not ctx.is_distributed:
        return [chunks[0]]
    dev = _backend_device(ctx)
    ref = chunks[0]
    send = [c.contiguous().to(dev) for c in chunks]
    sizes = torch.tensor([c.shape[0] for c in send], dtype=torch.int64, device=dev)
    recv_sizes = torch.zeros_like(sizes)
    dist.all_to_all_single(recv_sizes, sizes)
    tail = tuple(ref.shape[1:])
    inp = torch.cat(send, dim=0) if send else torch.zeros((0,) + tail, dtype=ref.dtype, device=dev)
    out = torch.empty((int(recv_sizes.sum().item()),) + tail, dtype=ref.dtype, device=dev)
    # one exchange of the payload on both backends (gloo implements all_to_all_single with
    # uneven splits for CPU tensors; RCCL for device tensors)
    dist.all_to_all_single(out, inp, output_split_sizes=recv_sizes.tolist(), input_split_sizes=sizes.tolist())
    return [p.to(ref.device) for p in torch.split(out, recv_sizes.tolist(), dim=0)]


def all_to_all_objects(objs: Sequence[Any]) -> List[Any]:
    ctx = get_context()
    if not ctx.is_distributed:
        return [objs[0]]
    gathered = all_gather_object(list(objs))
    return [g[ctx.rank] for g in gathered]


def check_equal_across_ranks(value: int, what: str) -> None:
    """All-reduce MIN and MAX to check a value agrees across ranks (``LogisticRegression.java:95-104``)."""
    ctx = get_context()
    if not ctx.is_distributed:
        return
    lo = all_reduce_scalar(float(value), "min")
    hi = all_reduce_scalar(float(value), "max")
    if lo != hi:
        raise ValueError("%s differs across ranks: min %s, max %s" % (what, lo, hi))


def barrier() -> None:
    ctx = get_context()
    if ctx.is_distributed:
        dist.barrier()
