"""Broadcast variables, keyed reduce, EndOfStreamWindows and LabeledPointWithWeight (reference
CORET/common/broadcast/BroadcastUtilsTest.java, CORET/common/datastream/DataStreamUtilsTest.java
shapes: every subtask sees every broadcast record; keyed reduce folds per key across subtasks)."""
import torch

from flink_ml_amd import Table, Vectors
from tests.spmd import run_spmd


def _bcast_worker(rank, world):
    from flink_ml_amd.parallel.broadcast import BroadcastContext, with_broadcast_stream

    part = Table.from_rows([(float(rank * 10 + i),) for i in range(rank + 1)], ["x"])
    model = Table.from_rows([(1.5,)], ["m"]).as_replicated()
    tens = torch.tensor([float(rank)])

    def fn(inputs, ctx):
        b = ctx.get_broadcast_variable("parts")
        m = ctx.get_broadcast_variable("model")
        t = ctx.get_broadcast_variable("tens")
        return (sorted(r[0] for r in b.rows()), m.num_rows, t.tolist(), inputs[0].num_rows)

    out = with_broadcast_stream([part], {"parts": part, "model": model, "tens": tens}, fn)
    # the registry is cleaned up after the call
    try:
        BroadcastContext.get("parts-%d" % rank)
        leaked = True
    except KeyError:
        leaked = False
    return out, leaked


def test_with_broadcast_stream_every_rank_sees_every_record():
    res = run_spmd(_bcast_worker, 3)
    expect = sorted([0.0, 10.0, 11.0, 20.0, 21.0, 22.0])
    for rank, (out, leaked) in enumerate(res):
        vals, mrows, tens, nin = out
        assert vals == expect
        assert mrows == 1  # replicated input is not multiplied by the world size
        assert tens == [0.0, 1.0, 2.0]
        assert nin == rank + 1  # the non-broadcast input stays the local partition
        assert not leaked


def _keyed_worker(rank, world):
    from flink_ml_amd.parallel.datastream import reduce_by_key

    pairs = [("a", rank + 1), ("b", 10 * (rank + 1))] + ([("c", 100)] if rank == 1 else [])
    return reduce_by_key(pairs, lambda x, y: x + y)


def test_reduce_by_key_across_ranks():
    res = run_spmd(_keyed_worker, 2)
    assert res[0] == res[1] == {"a": 3, "b": 30, "c": 100}


def test_end_of_stream_windows_single_window():
    from flink_ml_amd.common.window import EndOfStreamWindows
    from flink_ml_amd.parallel.datastream import window_all_and_process

    t = Table.from_rows([(float(i),) for i in range(7)], ["x"])
    out = window_all_and_process(t, EndOfStreamWindows.get(),
                                 lambda w: Table.from_rows([(float(w.num_rows),)], ["n"]))
    assert out.rows() == [(7.0,)]
    assert EndOfStreamWindows.get() is EndOfStreamWindows.get()


def test_labeled_point_with_weight_table_roundtrip():
    from flink_ml_amd.common.feature import LabeledPointWithWeight

    pts = [LabeledPointWithWeight(Vectors.dense(1.0, 2.0), 1.0, 0.5),
           LabeledPointWithWeight(Vectors.dense(3.0, 4.0), 0.0)]
    t = LabeledPointWithWeight.to_table(pts)
    back = LabeledPointWithWeight.from_table(t, weight_col="weight")
    assert [(p.get_label(), p.get_weight()) for p in back] == [(1.0, 0.5), (0.0, 1.0)]
    assert back[1].get_features() == Vectors.dense(3.0, 4.0)


def _a2a_worker(rank, world):
    import torch

    from flink_ml_amd.parallel import comm

    # rank r sends (r + 1) * (dst + 1) rows of width 3 to every dst, filled with 100 r + dst
    chunks = [torch.full(((rank + 1) * (dst + 1), 3), float(100 * rank + dst)) for dst in range(world)]
    got = comm.all_to_all_v(chunks)
    return [(tuple(g.shape), float(g[0, 0]) if g.numel() else None) for g in got]


def test_all_to_all_v_uneven_splits():
    res = run_spmd(_a2a_worker, 3)
    for dst, recv in enumerate(res):
        assert recv == [(((src + 1) * (dst + 1), 3), float(100 * src + dst)) for src in range(3)]


def _keyed_tensor_worker(rank, world):
    from flink_ml_amd.parallel.datastream import reduce_by_key_tensor

    g = torch.Generator().manual_seed(rank)
    keys = torch.randint(-20, 50, (500,), generator=g)
    vals = torch.randn((500, 3), generator=g, dtype=torch.float64)
    own = {op: reduce_by_key_tensor(keys, vals, op) for op in ("sum", "min", "max")}
    full = reduce_by_key_tensor(keys, vals, "sum", gather=True)
    # numpy across the result queue: torch tensors travel as shared-memory fds that vanish
    # once the worker exits
    npy = lambda kv: (kv[0].numpy(), kv[1].numpy())  # noqa: E731
    return keys.numpy(), vals.numpy(), {op: npy(kv) for op, kv in own.items()}, npy(full)


def test_reduce_by_key_tensor_across_ranks():
    from flink_ml_amd.parallel.datastream import key_owner

    world = 3
    res = [(torch.from_numpy(k), torch.from_numpy(v), {op: tuple(map(torch.from_numpy, kv)) for op, kv in own.items()},
            tuple(map(torch.from_numpy, full))) for k, v, own, full in run_spmd(_keyed_tensor_worker, world)]
    K = torch.cat([r[0] for r in res])
    V = torch.cat([r[1] for r in res])
    uk = torch.unique(K)
    for op, red in (("sum", lambda x: x.sum(0)), ("min", lambda x: x.min(0).values),
                    ("max", lambda x: x.max(0).values)):
        seen = []
        for rank, (_, _, own, _) in enumerate(res):
            k, v = own[op]
            assert torch.all(key_owner(k, world) == rank)  # each key reduced on its owner only
            for kk, vv in zip(k.tolist(), v):
                torch.testing.assert_close(vv, red(V[K == kk]))
            seen += k.tolist()
        assert sorted(seen) == uk.tolist()
    for _, _, _, (k, v) in res:  # gather=True: everyone has every key
        assert k.tolist() == uk.tolist()
        torch.testing.assert_close(v[3], V[K == uk[3]].sum(0))
