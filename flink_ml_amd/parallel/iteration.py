"""Iteration runtime: bounded / unbounded SPMD round loops with the reference's semantics.

Reference: ``flink-ml-iteration`` (``ITER/Iterations.java``, ``IterationBody.java``,
``IterationListener.java``, ``IterationConfig.java``, ``ReplayableDataStreamList.java``, head/tail/
coordinator operators). There the loop is a cyclic dataflow graph: records carry an epoch, a
head/tail pair closes the feedback edge inside one JVM, epoch watermarks flow in-band and an
operator coordinator aligns rounds globally and decides termination
(``SharedProgressAligner.java:277-300``).

MI355X-native replacement: every rank runs the *same* round loop in lockstep;
a round is one call of the body over the rank's partition (device tensors stay in HBM), the
feedback edge is a hand-over of Python/device objects (zero copy), epoch alignment is implicit,
and the termination decision is one all-reduce of two record counts. Semantics kept:

* epochs start at 0; records fed back become the next round's variables (epoch + 1);
* termination is never decided before round 0 completes; after round e the loop stops when the
  global number of fed-back variable records is 0, or when a termination-criteria stream is
  given and it produced no record in round e (``SharedProgressAligner.EpochStatus.isTerminated``);
* ``IterationListener.on_epoch_watermark_incremented(epoch, ctx, collector)`` fires on every
  registered listener at the end of each round, ``on_iteration_terminated`` once at the end;
  records they emit go to the collector's output (epoch = the watermark);
* data streams are passed every round when replayed (``ReplayableDataStreamList.replay``) and
  only in round 0 otherwise (the operator caches them, like ``ListStateWithCache``);
* ``OperatorLifeCycle.ALL_ROUND`` keeps one body instance for all rounds; ``PER_ROUND`` builds
  a fresh body (operator state reset) every round from a factory.
* Unbounded iterations consume an input stream of mini-batches and run until it ends.
* side outputs: ``context.output(tag, record)`` — from the body or from a listener callback
  (``IterationListener.Context.output``, ``IterationListener.java:66-73``) — is delivered as a
  named stream of the returned ``IterationResult`` (``get_side_output(tag)``), in emission order.
* Round-level checkpoints (bounded AND unbounded): a ``RoundCheckpointer`` persists (variables,
  epoch, outputs, side outputs) every N rounds; an unbounded run also records how many input
  batches it consumed and skips them on resume (the source replays from the start, like a
  checkpointed Flink source rewinding to its offset).
* Observability: each round is a roctx range (``FMLX_TRACE=1``) and, with
  ``FMLX_LOG_ROUNDS=1``, one structured JSON log line (rank, epoch, fed-back records, ms).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import Any, Callable, Iterable, Iterator, List, Optional, Sequence

import time

from . import comm
from ..utils import tracing


class OperatorLifeCycle(enum.Enum):
    ALL_ROUND = "ALL_ROUND"
    PER_ROUND = "PER_ROUND"


@dataclass
class IterationConfig:
    operator_life_cycle: OperatorLifeCycle = OperatorLifeCycle.ALL_ROUND
    # unbounded iterations: rounds per end-of-stream agreement. The ranks agree on how many
    # batches every rank has (one scalar all-reduce per ``agree_interval`` rounds, on up to that
    # many prefetched local batches) instead of once per batch; 0 = no agreement at all (the
    # caller guarantees equally long streams; the round counts are checked once at the end).
    # Semantics are unchanged: the iteration ends when the stream ends on any rank.
    agree_interval: int = 1

    @staticmethod
    def new_builder():
        return _ConfigBuilder()


class _ConfigBuilder:
    def __init__(self):
        self._lc = OperatorLifeCycle.ALL_ROUND
        self._agree = 1

    def set_operator_life_cycle(self, lc: OperatorLifeCycle):
        self._lc = lc
        return self

    def set_agree_interval(self, k: int):
        self._agree = int(k)
        return self

    def build(self) -> IterationConfig:
        return IterationConfig(self._lc, self._agree)


class DataStreamList(list):
    """A list of per-rank record collections (lists, Tables, tensors)."""

    @staticmethod
    def of(*streams) -> "DataStreamList":
        return DataStreamList(streams)

    def get(self, i: int):
        return self[i]


class IterationResult(DataStreamList):
    """The output streams of an iteration plus its side outputs by tag."""

    def __init__(self, outputs, side_outputs=None):
        super().__init__(outputs)
        self.side_outputs = dict(side_outputs or {})

    def get_side_output(self, tag: str) -> list:
        return list(self.side_outputs.get(tag, []))

    getSideOutput = get_side_output


class ReplayableDataStreamList:
    def __init__(self, replayed: Sequence, non_replayed: Sequence):
        self.replayed = list(replayed)
        self.non_replayed = list(non_replayed)

    @staticmethod
    def replay(*streams) -> "ReplayableDataStreamList":
        return ReplayableDataStreamList(streams, [])

    @staticmethod
    def not_replay(*streams) -> "ReplayableDataStreamList":
        return ReplayableDataStreamList([], streams)

    def and_not_replay(self, *streams) -> "ReplayableDataStreamList":
        return ReplayableDataStreamList(self.replayed, self.non_replayed + list(streams))


class Collector:
    def __init__(self):
        self.records: List[Any] = []

    def collect(self, record) -> None:
        self.records.append(record)


class IterationContext:
    """Passed to the body each round: epoch, rank info, listener registration, side outputs."""

    def __init__(self, epoch: int):
        self.epoch = epoch
        self.side_outputs = {}
        from .context import get_context

        c = get_context()
        self.rank, self.world_size = c.rank, c.world_size

    def output(self, tag: str, record) -> None:
        self.side_outputs.setdefault(tag, []).append(record)


class IterationListener:
    def on_epoch_watermark_incremented(self, epoch: int, context: IterationContext, collector: Collector) -> None:
        pass

    def on_iteration_terminated(self, context: IterationContext, collector: Collector) -> None:
        pass


@dataclass
class IterationBodyResult:
    feedback_variable_streams: Sequence
    output_streams: Sequence
    termination_criteria: Optional[Sequence] = None
    # listeners whose callbacks fire at the end of this round / at termination; each maps to the
    # index of the output stream its collector appends to (None → discarded)
    listeners: Sequence = field(default_factory=list)


class IterationBody:
    def process(self, variable_streams: DataStreamList, data_streams: DataStreamList,
                context: IterationContext) -> IterationBodyResult:
        raise NotImplementedError

    @staticmethod
    def for_each_round(streams, fn: Callable):
        """Per-round sub-graph (``IterationBody.forEachRound``): in the SPMD runtime every round
        already re-invokes the body, so this simply applies ``fn``."""
        return fn(streams)


def _count(stream) -> int:
    if stream is None:
        return 0
    try:
        return len(stream)
    except TypeError:
        return 1


class Iterations:
    @staticmethod
    def iterate_bounded_streams_until_termination(init_variables: Sequence, data: ReplayableDataStreamList,
                                                  config: IterationConfig, body,
                                                  max_rounds: Optional[int] = None,
                                                  checkpoint: Optional["RoundCheckpointer"] = None) -> DataStreamList:
        """Runs the body round by round; returns the collected output streams."""
        return _run_bounded(init_variables, data, config, body, max_rounds, checkpoint)

    @staticmethod
    def iterate_unbounded_streams(init_variables: Sequence, data_batches: Iterable, body,
                                  config: IterationConfig = None,
                                  checkpoint: Optional["RoundCheckpointer"] = None) -> DataStreamList:
        """One round per arriving mini-batch; terminates when the stream ends on any rank."""
        return _run_unbounded(init_variables, data_batches, config or IterationConfig(), body, checkpoint)

    iterateBoundedStreamsUntilTermination = iterate_bounded_streams_until_termination
    iterateUnboundedStreams = iterate_unbounded_streams


def _make_body(body, config, epoch):
    if config.operator_life_cycle == OperatorLifeCycle.PER_ROUND and callable(body) and not isinstance(
            body, IterationBody):
        return body()
    if config.operator_life_cycle == OperatorLifeCycle.PER_ROUND and hasattr(body, "fresh"):
        return body.fresh()
    if isinstance(body, IterationBody) or hasattr(body, "process"):
        return body
    return body()


def _merge_side(side: dict, ctx: IterationContext) -> None:
    for tag, recs in ctx.side_outputs.items():
        side.setdefault(tag, []).extend(recs)
    ctx.side_outputs = {}


def _emit_listener_records(result: IterationBodyResult, outputs: List[list], epoch: int, terminated: bool,
                           ctx: IterationContext):
    for item in (result.listeners or ()) if result is not None else ():
        listener, out_idx = item if isinstance(item, tuple) else (item, None)
        coll = Collector()
        if terminated:
            listener.on_iteration_terminated(ctx, coll)
        else:
            listener.on_epoch_watermark_incremented(epoch, ctx, coll)
        if out_idx is not None:
            outputs[out_idx].extend(coll.records)


def _run_bounded(init_variables, data, config, body_or_factory, max_rounds, checkpoint):
    variables = DataStreamList(init_variables)
    outputs: List[list] = []
    side: dict = {}
    epoch = 0
    if checkpoint is not None:
        restored = checkpoint.restore()
        if restored is not None:
            epoch, variables, outputs = restored["epoch"], DataStreamList(restored["variables"]), restored["outputs"]
            side = restored.get("side", {})
    body = _make_body(body_or_factory, config, epoch)
    last_result = None
    while True:
        if config.operator_life_cycle == OperatorLifeCycle.PER_ROUND:
            body = _make_body(body_or_factory, config, epoch)
        from .checkpoint import fault_point

        fault_point(epoch)
        ctx = IterationContext(epoch)
        streams = DataStreamList(list(data.replayed) + (list(data.non_replayed) if epoch == 0 else
                                                        [None] * len(data.non_replayed)))
        t0 = time.perf_counter()
        with tracing.range("iteration.round"):
            result = body.process(variables, streams, ctx)
            if not outputs:
                outputs = [[] for _ in result.output_streams]
            for i, o in enumerate(result.output_streams):
                if o is not None:
                    outputs[i].extend(o if isinstance(o, list) else [o])
            _emit_listener_records(result, outputs, epoch, False, ctx)
            _merge_side(side, ctx)
            n_feedback = sum(_count(s) for s in result.feedback_variable_streams)
            n_crit = _count(result.termination_criteria) if result.termination_criteria is not None else -1
            # the coordinator's alignment (SharedProgressAligner): global record counts decide
            tot, crit_tot = _global_counts(float(n_feedback), float(max(n_crit, 0)) if n_crit >= 0 else None)
        tracing.log_round(kind="bounded", rank=ctx.rank, epoch=epoch, feedback_records=int(tot),
                          criteria_records=None if crit_tot is None else int(crit_tot),
                          ms=round((time.perf_counter() - t0) * 1e3, 3))
        last_result = result
        epoch += 1
        if tot == 0 or crit_tot == 0 or (max_rounds is not None and epoch >= max_rounds):
            break
        variables = DataStreamList(result.feedback_variable_streams)
        if checkpoint is not None:
            checkpoint.maybe_save(epoch, variables, outputs, side=side)
    ctx = IterationContext(epoch)
    _emit_listener_records(last_result, outputs, epoch, True, ctx)
    _merge_side(side, ctx)
    return IterationResult(outputs, side)


def _global_counts(n_feedback: float, n_crit):
    """ONE all-reduce of [feedback records, criteria records] (instead of one per count)."""
    import torch

    from .context import get_context

    if not get_context().is_distributed:
        return n_feedback, n_crit
    t = torch.tensor([n_feedback, -1.0 if n_crit is None else n_crit], dtype=torch.float64)
    comm.all_reduce_sum(t)
    crit = None if n_crit is None else float(t[1])
    return float(t[0]), crit


def _run_unbounded(init_variables, data_batches, config, body_or_factory, checkpoint=None):
    variables = DataStreamList(init_variables)
    outputs: List[list] = []
    side: dict = {}
    epoch = 0
    it: Iterator = iter(data_batches)
    if checkpoint is not None:
        restored = checkpoint.restore()
        if restored is not None:
            epoch, variables, outputs = restored["epoch"], DataStreamList(restored["variables"]), restored["outputs"]
            side = restored.get("side", {})
            for _ in range(epoch):  # the batches those rounds consumed (the source rewinds)
                next(it, None)
    body = _make_body(body_or_factory, config, epoch)
    last_result = None
    from collections import deque

    from .checkpoint import fault_point

    K = max(0, int(getattr(config, "agree_interval", 1)))
    ready: deque = deque()  # prefetched local batches every rank is known to have
    agreed = 0              # rounds still covered by the last agreement
    ended = False
    last = False            # the last agreement covered fewer than K rounds: some stream ended

    def next_batch():
        nonlocal agreed, ended, last
        if K == 0:  # aligned streams: no per-round collective
            try:
                return next(it), True
            except StopIteration:
                return None, False
        if agreed == 0:
            if last:
                return None, False
            # prefetch up to K local batches, then one agreement on the common count
            while len(ready) < K and not ended:
                try:
                    ready.append(next(it))
                except StopIteration:
                    ended = True
            agreed = int(comm.all_reduce_scalar(float(len(ready)), "min"))
            last = agreed < K  # a rank came up short only because its stream ended
            if agreed == 0:
                return None, False
        agreed -= 1
        return ready.popleft(), True

    while True:
        batch, ok = next_batch()
        if not ok:
            break
        fault_point(epoch)
        if config.operator_life_cycle == OperatorLifeCycle.PER_ROUND:
            body = _make_body(body_or_factory, config, epoch)
        ctx = IterationContext(epoch)
        t0 = time.perf_counter()
        with tracing.range("iteration.round"):
            result = body.process(variables, DataStreamList([batch]), ctx)
            if not outputs:
                outputs = [[] for _ in result.output_streams]
            for i, o in enumerate(result.output_streams):
                if o is not None:
                    outputs[i].extend(o if isinstance(o, list) else [o])
            _emit_listener_records(result, outputs, epoch, False, ctx)
            _merge_side(side, ctx)
        tracing.log_round(kind="unbounded", rank=ctx.rank, epoch=epoch, ms=round((time.perf_counter() - t0) * 1e3, 3))
        variables = DataStreamList(result.feedback_variable_streams)
        last_result = result
        epoch += 1
        if checkpoint is not None:
            checkpoint.maybe_save(epoch, variables, outputs, side=side)
    if K == 0:
        lo, hi = comm.all_reduce_scalar(float(epoch), "min"), comm.all_reduce_scalar(float(epoch), "max")
        if lo != hi:
            raise RuntimeError("agree_interval=0 needs equally long streams: ranks ran %d..%d rounds" % (lo, hi))
    if last_result is not None:
        ctx = IterationContext(epoch)
        _emit_listener_records(last_result, outputs, epoch, True, ctx)
        _merge_side(side, ctx)
    return IterationResult(outputs, side)


class TerminateOnMaxIter(IterationListener):
    """Criteria stream helper (``common/iteration/TerminateOnMaxIter.java:47-52``): emits a record
    while ``epoch + 1 < max_iter``."""

    def __init__(self, max_iter: int):
        self.max_iter = max_iter

    def criteria(self, epoch: int) -> list:
        return [0] if epoch + 1 < self.max_iter else []


class TerminateOnMaxIterOrTol(IterationListener):
    """``TerminateOnMaxIterOrTol.java:54-68``: emits while ``epoch+1 < maxIter and loss > tol``."""

    def __init__(self, max_iter: int = 2 ** 31 - 1, tol: float = 0.0):
        self.max_iter = max_iter
        self.tol = tol

    def criteria(self, epoch: int, loss: float) -> list:
        return [0] if (epoch + 1 < self.max_iter and loss > self.tol) else []


class ForwardInputsOfLastRound(IterationListener):
    """Buffers the records of the current round and forwards only the last round's on
    termination (``ForwardInputsOfLastRound.java:38-59``)."""

    def __init__(self):
        self.buffer = []

    def add(self, records) -> None:
        self.buffer = list(records)

    def on_epoch_watermark_incremented(self, epoch, context, collector):
        pass

    def on_iteration_terminated(self, context, collector):
        for r in self.buffer:
            collector.collect(r)


class RoundCheckpointer:
    """Round-level checkpoint of an iteration: the variables fed back into the next round and the
    outputs collected so far are saved through ``parallel.checkpoint`` every ``interval`` rounds
    and restored on restart (the analogue of the head operator's checkpointed feedback)."""

    def __init__(self, name: str = "iteration"):
        from .checkpoint import AlgorithmCheckpoint

        self._ck = AlgorithmCheckpoint(name)

    def restore(self):
        r = self._ck.restore()
        if r is None:
            return None
        epoch, st = r
        return {"epoch": epoch, "variables": st["variables"], "outputs": st["outputs"], "side": st.get("side", {})}

    def maybe_save(self, epoch: int, variables, outputs, side=None) -> None:
        self._ck.maybe_save(epoch, lambda: {"variables": list(variables), "outputs": [list(o) for o in outputs],
                                            "side": {k: list(v) for k, v in (side or {}).items()}})