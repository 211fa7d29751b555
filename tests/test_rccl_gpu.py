"""The RCCL (``nccl`` backend) code path on a one-GPU host: ``FMLX_FORCE_PG=1`` creates a real
process group at WORLD_SIZE=1 on the GPU, so every collective of the distributed trainers runs
through RCCL exactly as on eight GPUs (an identity sum at one rank) — including all-reduces
captured into hipGraphs, and the fallback taken when the xGMI exchange fails its self-test.
Reference analogue: ``flink-ml-core/src/test/java/org/apache/flink/ml/common/datastream/
AllReduceImplTest.java:47-75`` (the all-reduce exercised through the real network stack).

Every worker runs in a spawned process (its own process group); results are compared with the
same computation in the parent process, which has no process group."""
import numpy as np
import pytest
import torch

from tests.spmd import run_spmd

pytestmark = pytest.mark.gpu

RCCL = {"FMLX_DEVICE": "cuda:0", "FMLX_FORCE_PG": "1", "FMLX_XGMI": "0"}


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _sparse_data(seed=21, n=20_000, d=1_000_000, nnz=32):
    from flink_ml_amd.table import SparseColumn

    g = torch.Generator(device="cpu").manual_seed(seed)
    idx = torch.randint(0, d, (n, nnz), generator=g).sort(dim=1).values  # a repeated index adds twice
    vals = torch.rand((n, nnz), generator=g, dtype=torch.float32)
    indptr = torch.arange(0, n * nnz + 1, nnz, dtype=torch.int64)
    y = (vals[:, :4].sum(1) > 2).to(torch.float32)
    return SparseColumn(indptr, idx.reshape(-1).to(torch.int32), vals.reshape(-1), d), y


def _fit_svc_sparse(graph: bool):
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer

    X, y = _sparse_data()
    X = X.to("cuda:0")
    sgd = SGD(max_iter=12, learning_rate=0.1, global_batch_size=4_000, tol=0.0)
    tr = DeviceGlmTrainer(sgd, np.zeros(X.size), X, y.cuda(), None, "hinge", use_graph=graph)
    tr.rounds_per_graph = 4
    tr.bkt_graph_min_iters = 0  # capture even this short bucket-round fit
    coef = tr.fit()
    return tr, coef


def _fit_lr_dense(graph: bool):
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer

    g = torch.Generator(device="cpu").manual_seed(5)
    n, d = 60_000, 1000
    X = torch.rand((n, d), generator=g).to(torch.bfloat16)
    y = torch.randint(0, 2, (n,), generator=g).to(torch.float32)
    sgd = SGD(max_iter=9, learning_rate=0.1, global_batch_size=20_000, tol=0.0)
    tr = DeviceGlmTrainer(sgd, np.zeros(d), X.cuda(), y.cuda(), None, "logistic", use_graph=graph)
    tr.rounds_per_graph = 4
    return tr, tr.fit()


def _glm_worker(rank, world):
    from flink_ml_amd.common.optimizer import SGD  # noqa: F401
    from flink_ml_amd.ops import glm as gk
    from flink_ml_amd.parallel import xgmi
    from flink_ml_amd.parallel.context import get_context

    ctx = get_context()
    assert ctx.is_distributed and ctx.backend == "nccl" and ctx.world_size == 1
    assert xgmi.collective_path() == "nccl"
    out = {}
    tr, c = _fit_svc_sparse(graph=True)
    assert tr.distributed and tr.mode == gk.TAIL_FEEDBACK and tr.use_graph and tr.bkt is not None
    assert tr.feedback.numel() == 1_000_002  # 4 MB: beyond the xGMI one-shot cap in any case
    assert len(tr.graphs) > 0  # the RCCL all-reduce was captured into hipGraphs and replayed
    out["svc"] = (c, tr.rounds_executed())
    tr, c = _fit_lr_dense(graph=True)
    assert tr.mode == gk.TAIL_FEEDBACK and tr.use_graph and len(tr.graphs) > 0
    out["lr"] = (c, tr.rounds_executed())
    return out


def test_glm_rounds_on_rccl_with_hipgraph():
    """TAIL_FEEDBACK rounds whose RCCL all-reduce of the (d+2) feedback is captured into hipGraphs:
    the sparse LinearSVC path (1M-wide feedback) and the dense LR path, against the same fits
    without a process group (fused 1-GPU kernels)."""
    _need_gpu()
    (res,) = run_spmd(_glm_worker, 1, env=RCCL, backend=None, timeout=300)
    tr, ref = _fit_svc_sparse(graph=True)
    c, rounds = res["svc"]
    assert rounds == tr.rounds_executed() == 12
    assert np.allclose(c, ref, rtol=1e-5, atol=1e-6), np.abs(c - ref).max()
    tr, ref = _fit_lr_dense(graph=True)
    c, rounds = res["lr"]
    assert rounds == 9
    assert np.allclose(c, ref, rtol=2e-4, atol=2e-6), np.abs(c - ref).max()


def _kmeans_online_worker(rank, world):
    from flink_ml_amd.ops import kmeans as kk
    from flink_ml_amd.parallel import xgmi

    assert xgmi.collective_path() == "nccl"
    assert kk.GROUP_SORT  # the default stable counting sort: bit-reproducible sums
    return {"kmeans": _kmeans_fit(), "online": _online_fit()}


def _kmeans_fit():
    from flink_ml_amd.models.kmeans import kmeans_lloyd

    g = torch.Generator(device="cpu").manual_seed(3)
    X = torch.rand((200_000, 32), generator=g).cuda()
    init = X[:64].double().cpu().numpy()
    out = kmeans_lloyd(X, init, 6, "euclidean")
    return np.asarray(out[0] if isinstance(out, tuple) else out)


def _online_fit():
    from flink_ml_amd import Table
    from flink_ml_amd.lib.classification.logisticregression import OnlineLogisticRegression
    from flink_ml_amd.linalg import Vectors
    from flink_ml_amd.stream import StreamTable

    dim, gb = 64, 4096
    g = torch.Generator(device="cpu").manual_seed(17)
    X = torch.rand((gb * 6, dim), generator=g).cuda()
    y = (X[:, :4].sum(1) > 2).double()
    init = Table.from_rows([(Vectors.dense(np.zeros(dim)), 0)], ["coefficient", "modelVersion"])
    model = OnlineLogisticRegression().set_global_batch_size(gb).set_initial_model_data(init).fit(
        StreamTable.from_table(Table({"features": X, "label": y}), gb))
    stream = model._stream
    n = 0
    while n < 6 and stream.pull(block=True):
        n += 1
    stream.flush()
    ver = model.model_data_rows()[0]  # (coefficient, modelVersion) of the newest version
    return np.asarray(ver[0].values, dtype=np.float64), n


def test_kmeans_and_online_lr_on_rccl(monkeypatch):
    """KMeans (centroid all-reduce) and OnlineLogisticRegression (FTRL payload all-reduce) with the
    xGMI exchange off: every collective is an RCCL all-reduce; same results as without a group."""
    _need_gpu()
    (res,) = run_spmd(_kmeans_online_worker, 1, env=RCCL, backend=None, timeout=300)
    ref_k = _kmeans_fit()
    assert np.allclose(res["kmeans"], ref_k, rtol=1e-5, atol=1e-6)
    ref_o, n = _online_fit()
    got_o, n2 = res["online"]
    assert n == n2 == 6
    assert np.allclose(got_o, ref_o, rtol=1e-5, atol=1e-7), np.abs(got_o - ref_o).max()


def _fallback_worker(rank, world):
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk
    from flink_ml_amd.parallel import comm, xgmi

    out = {"path": xgmi.collective_path(), "xg": xgmi.get() is not None}
    t = torch.full((1000,), 3.0, device="cuda:0")
    comm.all_reduce_sum(t)
    out["sum_ok"] = bool(torch.all(t == 3.0).item())
    g = torch.Generator(device="cpu").manual_seed(2)
    X = torch.rand((8_000, 256), generator=g).cuda()
    y = torch.randint(0, 2, (8_000,), generator=g).to(torch.float32).cuda()
    tr = DeviceGlmTrainer(SGD(max_iter=5, learning_rate=0.1, global_batch_size=2_000, tol=0.0), np.zeros(256), X, y,
                          None, "logistic")
    out["mode"] = tr.mode
    out["coef"] = tr.fit()
    out["tail_feedback"] = gk.TAIL_FEEDBACK
    out["tail_xgmi"] = gk.TAIL_XGMI
    return out


@pytest.mark.parametrize("inject", [False, True])
def test_xgmi_self_test_failure_falls_back_to_rccl(inject):
    """With the exchange enabled, a failing xGMI self-test (injected) must leave every collective
    on RCCL — decided collectively — and the trainer in TAIL_FEEDBACK mode; without the injection
    the one-rank exchange comes up and the fused round runs its in-kernel exchange. Both fits
    agree."""
    _need_gpu()
    env = dict(RCCL, FMLX_XGMI="1")
    if inject:
        env["FMLX_XGMI_INJECT_FAIL"] = "1"
    (res,) = run_spmd(_fallback_worker, 1, env=env, backend=None, timeout=300)
    assert res["sum_ok"]
    if inject:
        assert res["path"] == "nccl" and not res["xg"] and res["mode"] == res["tail_feedback"]
    else:
        assert res["path"] == "xgmi" and res["xg"] and res["mode"] == res["tail_xgmi"]
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer

    g = torch.Generator(device="cpu").manual_seed(2)
    X = torch.rand((8_000, 256), generator=g).cuda()
    y = torch.randint(0, 2, (8_000,), generator=g).to(torch.float32).cuda()
    ref = DeviceGlmTrainer(SGD(max_iter=5, learning_rate=0.1, global_batch_size=2_000, tol=0.0), np.zeros(256), X, y,
                           None, "logistic").fit()
    assert np.allclose(res["coef"], ref, rtol=1e-4, atol=1e-6)
