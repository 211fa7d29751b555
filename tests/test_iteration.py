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


def test_side_outputs_from_body_and_listeners():
    """``Context.output(tag, record)`` (IterationListener.java:66-73) from the body and from the
    listener callbacks arrives as a named side-output stream, in emission order."""

    class L(IterationListener):
        def on_epoch_watermark_incremented(self, epoch, context, collector):
            context.output("wm", ("wm", epoch))

        def on_iteration_terminated(self, context, collector):
            context.output("wm", ("done", context.epoch))
            collector.collect("final")

    class B(IterationBody):
        def __init__(self):
            self.listener = L()

        def process(self, variables, data, ctx):
            ctx.output("body", ctx.epoch * 10)
            fb = [variables[0][0] + 1] if ctx.epoch < 2 else []
            return IterationBodyResult([fb], [[ctx.epoch]], listeners=[(self.listener, 0)])

    out = Iterations.iterate_bounded_streams_until_termination([[0]], ReplayableDataStreamList.replay([1]),
                                                               IterationConfig(), B())
    assert out[0] == [0, 1, 2, "final"]
    assert out.get_side_output("body") == [0, 10, 20]
    assert out.get_side_output("wm") == [("wm", 0), ("wm", 1), ("wm", 2), ("done", 3)]
    assert out.getSideOutput("missing") == []

    class U(IterationBody):
        def process(self, variables, data, ctx):
            ctx.output("seen", sum(data[0]))
            return IterationBodyResult([variables[0]], [[]])

    res = Iterations.iterate_unbounded_streams([[0]], iter([[1, 2], [3]]), U())
    assert res.get_side_output("seen") == [3, 3]


def _unbounded_ck(rank, world, ck_dir, attempt, fail_round):
    import os

    os.environ["FMLX_ATTEMPT"] = str(attempt)
    from flink_ml_amd.parallel import checkpoint as ckpt
    from flink_ml_amd.parallel.comm import all_reduce_scalar
    from flink_ml_amd.parallel.iteration import RoundCheckpointer

    ckpt.clear_faults()
    ckpt.enable(ck_dir, interval=2)
    if fail_round is not None:
        ckpt.inject(ckpt.FailAfter(fail_round, rank=0, on_attempt=0))

    class Acc(IterationBody):
        def process(self, variables, data, ctx):
            model = variables[0][0] + all_reduce_scalar(float(sum(data[0])), "sum")
            ctx.output("versions", ctx.epoch)
            return IterationBodyResult([[model]], [[model]])

    batches = [[rank * 100 + i, i] for i in range(9)]  # a replayable source: the same batches again
    out = Iterations.iterate_unbounded_streams([[0.0]], iter(batches), Acc(), checkpoint=RoundCheckpointer("online"))
    return out[0], out.get_side_output("versions")


def test_unbounded_iteration_failover_resumes_exactly(tmp_path):
    """An unbounded (online) iteration checkpoints every 2 batches; after an injected failure at
    batch 5 the restarted job skips the consumed batches and ends with the uninterrupted result."""
    clean = run_spmd(_unbounded_ck, 2, str(tmp_path / "clean"), 0, None)
    ck = str(tmp_path / "ck")
    with pytest.raises(RuntimeError, match="injected failure"):
        run_spmd(_unbounded_ck, 2, ck, 0, 5)
    resumed = run_spmd(_unbounded_ck, 2, ck, 1, 5)
    for (m0, v0), (m1, v1) in zip(clean, resumed):
        assert m0 == m1 and v0 == v1 == list(range(9))


def test_round_logs_are_structured_json(capsys):
    """FMLX_LOG_ROUNDS: one JSON record per round from the iteration runtime and the SGD trainer."""
    import io
    import json

    from flink_ml_amd import Table
    from flink_ml_amd.models import LogisticRegression
    from flink_ml_amd.utils import tracing

    sink = io.StringIO()
    tracing.log_rounds(True, sink)
    try:
        Iterations.iterate_bounded_streams_until_termination([[0]], ReplayableDataStreamList.replay(list(range(10))),
                                                             IterationConfig(), SumBody(3))
        X = torch.rand(200, 4, dtype=torch.float64)
        LogisticRegression().set_max_iter(4).set_global_batch_size(50).set_tol(0.0).fit(
            Table({"features": X, "label": (X[:, 0] > 0.5).double()}, num_rows=200))
    finally:
        tracing.log_rounds(False)
    recs = [json.loads(l) for l in sink.getvalue().splitlines()]
    it = [r for r in recs if r["kind"] == "bounded"]
    sgd = [r for r in recs if r["kind"] == "sgd"]
    assert [r["epoch"] for r in it] == [0, 1, 2] and all("ms" in r and r["rank"] == 0 for r in it)
    assert [r["epoch"] for r in sgd] == [0, 1, 2, 3] and all(r["weight"] == 50.0 and r["loss"] > 0 for r in sgd)


def _spmd_unbounded_agree(rank, world, k, counts):
    from flink_ml_amd.parallel import comm

    calls = {"n": 0}
    orig = comm.all_reduce_scalar

    def counting(x, op="sum", **kw):
        calls["n"] += 1
        return orig(x, op, **kw)

    comm.all_reduce_scalar = counting

    class B(IterationBody):
        def process(self, variables, data, ctx):
            model = variables[0][0] + sum(data[0])
            return IterationBodyResult([[model]], [[model]])

    batches = [[rank * 100 + i] for i in range(counts[rank])]
    cfg = IterationConfig.new_builder().set_agree_interval(k).build()
    try:
        out = Iterations.iterate_unbounded_streams([[0]], iter(batches), B(), config=cfg)
    finally:
        comm.all_reduce_scalar = orig
    return out[0], calls["n"]


@pytest.mark.parametrize("k", [1, 4, 0])
def test_unbounded_agreement_interval(k):
    """the end-of-stream agreement runs once per ``agree_interval`` rounds (0 =
    never during the run) and the iteration still stops when the shortest stream ends."""
    counts = [10, 10] if k == 0 else [10, 7]
    res = run_spmd(_spmd_unbounded_agree, 2, k, counts)
    n = min(counts)
    for rank, (out, calls) in enumerate(res):
        assert len(out) == n
        assert out[-1] == sum(rank * 100 + i for i in range(n))
        if k == 1:
            assert calls == n + 1
        elif k == 4:
            assert calls == -(-n // 4) + (1 if n % 4 == 0 else 0)
        else:
            assert calls == 2  # the final min/max check of the round counts
