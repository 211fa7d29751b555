"""Iteration runtime semantics (reference ITT/Bounded{AllRound,PerRound}StreamIterationITCase,
UnboundedStreamIterationITCase, ITERT/operator/coordinator/SharedProgressAlignerTest) and
DataStreamUtils equivalents (CORET/common/datastream/*Test)."""
import numpy as np
import pytest
import torch

from flink_ml_amd.parallel import datastream as ds
from flink_ml_amd.parallel.iteration import (Collector, DataStreamList, ForwardInputsOfLastRound, IterationBody,
                                             IterationBodyResult, IterationConfig, IterationListener, Iterations,
                                             OperatorLifeCycle, ReplayableDataStreamList, TerminateOnMaxIter)
from tests.spmd import run_spmd


class SumBody(IterationBody):
    """Variable = round counter; data = 0..999 (cached in round 0 unless replayed); every round
    outputs the sum of the data — the reference IT's per-round statistic."""

    def __init__(self, max_round, use_criteria=True):
        self.cache = None
        self.max_round = max_round
        self.use_criteria = use_criteria
        self.rounds_seen = 0

    def process(self, variables, data, ctx):
        if data[0] is not None:
            self.cache = list(data[0])
        self.rounds_seen += 1
        total = sum(self.cache)
        feedback = [v + 1 for v in variables[0]] if ctx.epoch + 1 < self.max_round or self.use_criteria else []
        crit = TerminateOnMaxIter(self.max_round).criteria(ctx.epoch) if self.use_criteria else None
        return IterationBodyResult([feedback], [[(ctx.epoch, total)]], crit)


def test_bounded_all_round_with_criteria():
    body = SumBody(5)
    out = Iterations.iterate_bounded_streams_until_termination(
        [[0]], ReplayableDataStreamList.not_replay(list(range(1000))), IterationConfig(), body)
    assert [e for e, _ in out[0]] == [0, 1, 2, 3, 4]
    assert all(s == 999 * 1000 // 2 for _, s in out[0])
    assert body.rounds_seen == 5


def test_terminates_when_feedback_empty():
    body = SumBody(3, use_criteria=False)
    out = Iterations.iterate_bounded_streams_until_termination(
        [[0]], ReplayableDataStreamList.replay(list(range(10))), IterationConfig(), body)
    assert len(out[0]) == 3


def test_never_terminates_before_round_zero_runs():
    body = SumBody(0)
    out = Iterations.iterate_bounded_streams_until_termination(
        [[0]], ReplayableDataStreamList.not_replay([1]), IterationConfig(), body)
    assert len(out[0]) == 1


class Listener(IterationListener):
    def __init__(self):
        self.epochs = []

    def on_epoch_watermark_incremented(self, epoch, context, collector):
        self.epochs.append(epoch)
        collector.collect(("wm", epoch))

    def on_iteration_terminated(self, context, collector):
        collector.collect(("terminated", None))


def test_listener_events_and_per_round_lifecycle():
    created = []

    class PerRound(IterationBody):
        def __init__(self):
            created.append(self)
            self.lst = Listener()

        def process(self, variables, data, ctx):
            crit = TerminateOnMaxIter(4).criteria(ctx.epoch)
            return IterationBodyResult([variables[0]], [[]], crit, listeners=[(self.lst, 0)])

    cfg = IterationConfig.new_builder().set_operator_life_cycle(OperatorLifeCycle.PER_ROUND).build()
    out = Iterations.iterate_bounded_streams_until_termination([[1]], ReplayableDataStreamList.replay([0]), cfg,
                                                               PerRound)
    assert out[0] == [("wm", 0), ("wm", 1), ("wm", 2), ("wm", 3), ("terminated", None)]
    assert len(created) >= 4  # a fresh operator every round


def test_forward_inputs_of_last_round():
    fwd = ForwardInputsOfLastRound()

    class B(IterationBody):
        def process(self, variables, data, ctx):
            fwd.add([ctx.epoch * 10])
            return IterationBodyResult([variables[0]], [[]], TerminateOnMaxIter(3).criteria(ctx.epoch),
                                       listeners=[(fwd, 0)])

    out = Iterations.iterate_bounded_streams_until_termination([[0]], ReplayableDataStreamList.replay([0]),
                                                               IterationConfig(), B())
    assert out[0] == [20]


def test_unbounded_iteration():
    class B(IterationBody):
        def process(self, variables, data, ctx):
            model = variables[0][0] + sum(data[0])
            return IterationBodyResult([[model]], [[model]])

    out = Iterations.iterate_unbounded_streams([[0]], iter([[1, 2], [3], [4, 5]]), B())
    assert out[0] == [3, 6, 15]


def _spmd_iteration(rank, world):
    body = SumBody(4)
    data = list(range(rank, 1000, world))
    out = Iterations.iterate_bounded_streams_until_termination(
        [[0]], ReplayableDataStreamList.not_replay(data), IterationConfig(), body)
    return [s for _, s in out[0]]


def test_bounded_iteration_four_ranks():
    res = run_spmd(_spmd_iteration, 4)
    totals = [sum(r[e] for r in res) for e in range(4)]
    assert totals == [999 * 1000 // 2] * 4


# ---------------------------------------------------------------- DataStreamUtils
class SumCount(ds.AggregateFunction):
    def create_accumulator(self):
        return [0, 0]

    def add(self, v, acc):
        return [acc[0] + v, acc[1] + 1]

    def merge(self, a, b):
        return [a[0] + b[0], a[1] + b[1]]

    def get_result(self, acc):
        return acc[0] / acc[1]


def _spmd_datastream(rank, world):
    vals = list(range(rank * 10, rank * 10 + 10))
    t = torch.arange(8, dtype=torch.float64) * (rank + 1)
    r = ds.all_reduce_sum(t.clone())
    red = ds.reduce(sum(vals), lambda a, b: a + b)
    agg = ds.aggregate(vals, SumCount())
    samp = ds.sample(vals, 5, 42)
    batches = list(ds.generate_batch_data(iter(range(100)), 10))
    return r.tolist(), red, agg, samp, [len(b) for b in batches]


def test_datastream_utils_four_ranks():
    res = run_spmd(_spmd_datastream, 4)
    for r, red, agg, samp, blens in res:
        assert r == (torch.arange(8, dtype=torch.float64) * 10).tolist()
        assert red == sum(range(40)) and agg == 19.5
        assert samp == res[0][3] and len(samp) == 5
    assert res[0][4][0] == 3 and res[3][4][0] == 2  # 10 split over 4 ranks: 3,3,2,2


def test_sample_small_input_keeps_all():
    assert sorted(ds.sample([1, 2, 3], 5, 0)) == [1, 2, 3]


def test_window_all_and_process():
    from flink_ml_amd import Table
    from flink_ml_amd.common.window import CountTumblingWindows, GlobalWindows

    t = Table({"x": torch.arange(10, dtype=torch.float64)})
    out = ds.window_all_and_process(t, CountTumblingWindows.of(4), lambda w: Table({"s": w.column("x").sum()[None]}))
    assert out.column("s").tolist() == [6.0, 22.0]
    out = ds.window_all_and_process(t, GlobalWindows.get_instance(), lambda w: Table({"s": w.column("x").sum()[None]}))
    assert out.column("s").tolist() == [45.0]
