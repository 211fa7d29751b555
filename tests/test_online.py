"""OnlineLogisticRegression / OnlineKMeans (reference LIBT/classification/OnlineLogisticRegressionTest.java,
LIBT/clustering/OnlineKMeansTest.java): goldens, InMemorySource streaming, model versions & gauge."""
import numpy as np
import pytest
import torch

from flink_ml_amd import Table, Vectors
from flink_ml_amd.models import OnlineKMeans, OnlineKMeansModel, OnlineLogisticRegression
from flink_ml_amd.models.online import generate_random_kmeans_model_data
from flink_ml_amd.stream import InMemorySource, StreamTable
from flink_ml_amd.utils.tracing import MetricGroup
from tests.spmd import run_spmd

TRAIN1 = [(Vectors.dense(0.1, 2.), 0.), (Vectors.dense(0.2, 2.), 0.), (Vectors.dense(0.3, 2.), 0.),
          (Vectors.dense(0.4, 2.), 0.), (Vectors.dense(0.5, 2.), 0.), (Vectors.dense(11., 12.), 1.),
          (Vectors.dense(12., 11.), 1.), (Vectors.dense(13., 12.), 1.), (Vectors.dense(14., 12.), 1.),
          (Vectors.dense(15., 12.), 1.)]
TRAIN2 = [(Vectors.dense(0.2, 3.), 0.), (Vectors.dense(0.8, 1.), 0.), (Vectors.dense(0.7, 1.), 0.),
          (Vectors.dense(0.6, 2.), 0.), (Vectors.dense(0.2, 2.), 0.), (Vectors.dense(14., 17.), 1.),
          (Vectors.dense(15., 10.), 1.), (Vectors.dense(16., 16.), 1.), (Vectors.dense(17., 10.), 1.),
          (Vectors.dense(18., 13.), 1.)]
PREDICT = [(Vectors.dense(0.8, 2.7), 0.0), (Vectors.dense(15.5, 11.2), 1.0)]
EXP1 = sorted([[0.04481034155642882, 0.9551896584435712], [0.5353966697318491, 0.4646033302681509]])
EXP2 = sorted([[0.013104324065967066, 0.9868956759340329], [0.5095144380001769, 0.49048556199982307]])

ONE = [1.0, 1.0, 1.0]
S1 = [(Vectors.sparse(10, [1, 3, 4], ONE), 0., 1.0), (Vectors.sparse(10, [0, 2, 3], ONE), 0., 1.4),
      (Vectors.sparse(10, [0, 3, 4], ONE), 0., 1.3), (Vectors.sparse(10, [2, 3, 4], ONE), 0., 1.4),
      (Vectors.sparse(10, [1, 3, 4], ONE), 0., 1.6), (Vectors.sparse(10, [6, 7, 8], ONE), 1., 1.8),
      (Vectors.sparse(10, [6, 8, 9], ONE), 1., 1.9), (Vectors.sparse(10, [5, 8, 9], ONE), 1., 1.0),
      (Vectors.sparse(10, [5, 6, 7], ONE), 1., 1.1)]
S2 = [(Vectors.sparse(10, [1, 2, 4], ONE), 0., 1.0), (Vectors.sparse(10, [2, 3, 4], ONE), 0., 1.3),
      (Vectors.sparse(10, [0, 2, 4], ONE), 0., 1.4), (Vectors.sparse(10, [1, 3, 4], ONE), 0., 1.0),
      (Vectors.sparse(10, [6, 7, 9], ONE), 1., 1.6), (Vectors.sparse(10, [7, 8, 9], ONE), 1., 1.8),
      (Vectors.sparse(10, [5, 7, 9], ONE), 1., 1.0), (Vectors.sparse(10, [5, 6, 7], ONE), 1., 1.5),
      (Vectors.sparse(10, [5, 8, 9], ONE), 1., 1.0)]
SPRED = [(Vectors.sparse(10, [1, 3, 5], ONE), 0.), (Vectors.sparse(10, [5, 8, 9], ONE), 1.)]
SEXP1 = sorted([[0.4452309884735286, 0.5547690115264714], [0.5105551725414953, 0.4894448274585047]])
SEXP2 = sorted([[0.40310431554310666, 0.5968956844568933], [0.5249618837373886, 0.4750381162626114]])


def _raw(out):
    # the reference compares predictions as an unordered collection
    return sorted(r[3].values.tolist() for r in out.rows())


def test_params():
    m = OnlineLogisticRegression()
    assert m.get_alpha() == 0.1 and m.get_beta() == 0.1 and m.get_global_batch_size() == 32
    assert m.get_model_version_col() == "modelVersion" and m.get_batch_strategy() == "count"


def test_dense_fit_and_predict_streaming():
    src = InMemorySource()
    init = Table.from_rows([(Vectors.dense(0.41233679404769874, -0.18088118293232122), 0)],
                           ["coefficient", "modelVersion"])
    model = (OnlineLogisticRegression().set_reg(0.2).set_elastic_net(0.5).set_global_batch_size(10)
             .set_initial_model_data(init).fit(src))
    pred = Table.from_rows(PREDICT, ["features", "label"])
    src.add_rows(TRAIN1, ["features", "label"])
    out = model.transform(pred)[0]
    assert np.allclose(_raw(out), EXP1, atol=1e-7)
    assert out.column("modelVersion").tolist() == [1, 1]
    assert model.model_data_version() == 1
    src.add_rows(TRAIN2, ["features", "label"])
    out = model.transform(pred)[0]
    assert np.allclose(_raw(out), EXP2, atol=1e-7)
    assert model.model_data_version() == 2
    assert any(v == 2 for v in MetricGroup.find("modelDataVersion").values())


def test_sparse_fit_and_predict():
    init = Table.from_rows([(Vectors.dense(*([0.01] * 10)), 0)], ["coefficient", "modelVersion"])
    src = InMemorySource()
    model = (OnlineLogisticRegression().set_reg(0.2).set_elastic_net(0.5).set_global_batch_size(9)
             .set_initial_model_data(init).fit(src))
    pred = Table.from_rows(SPRED, ["features", "label"])
    src.add_rows([r[:2] for r in S1], ["features", "label"])
    out = model.transform(pred)[0]
    assert np.allclose(_raw(out), SEXP1, atol=1e-7)
    src.add_rows([r[:2] for r in S2], ["features", "label"])
    out = model.transform(pred)[0]
    assert np.allclose(_raw(out), SEXP2, atol=1e-7)
    src.close()


def test_model_data_stream_and_save_load(tmp_path):
    init = Table.from_rows([(Vectors.dense(0.41233679404769874, -0.18088118293232122), 0)],
                           ["coefficient", "modelVersion"])
    est = (OnlineLogisticRegression().set_reg(0.2).set_elastic_net(0.5).set_global_batch_size(10)
           .set_initial_model_data(init))
    model = est.fit(Table.from_rows(TRAIN1 + TRAIN2, ["features", "label"]))
    versions = [t.rows()[0][1] for t in model.get_model_data()[0]]
    assert versions == [1, 2]
    p = str(tmp_path / "olr")
    model.save(p)
    from flink_ml_amd.models import OnlineLogisticRegressionModel

    loaded = OnlineLogisticRegressionModel.load(p)
    out = loaded.transform(Table.from_rows(PREDICT, ["features", "label"]))[0]
    assert np.allclose(_raw(out), EXP2, atol=1e-7)
    est.save(str(tmp_path / "est"))
    assert OnlineLogisticRegression.load(str(tmp_path / "est")).get_reg() == 0.2


def _spmd_olr(rank, world):
    init = Table.from_rows([(Vectors.dense(0.41233679404769874, -0.18088118293232122), 0)],
                           ["coefficient", "modelVersion"])
    train = Table.from_rows(TRAIN1 + TRAIN2, ["features", "label"])
    # global batch 10 → each rank's share; feed each rank the rows of each global batch it owns
    b = 10 // world + (1 if 10 % world > rank else 0)
    off = sum(10 // world + (1 if 10 % world > r else 0) for r in range(rank))
    local = Table.concat([train.slice(off, off + b), train.slice(10 + off, 10 + off + b)])
    model = (OnlineLogisticRegression().set_reg(0.2).set_elastic_net(0.5).set_global_batch_size(10)
             .set_initial_model_data(init).fit(local))
    out = model.transform(Table.from_rows(PREDICT, ["features", "label"]))[0]
    return _raw(out)


def test_online_lr_four_ranks():
    for raw in run_spmd(_spmd_olr, 4):
        assert np.allclose(raw, EXP2, atol=1e-7)


# ---------------------------------------------------------------- OnlineKMeans
def test_online_kmeans_streaming():
    init = generate_random_kmeans_model_data(2, 2, 0.0, 0)
    src = InMemorySource()
    model = OnlineKMeans().set_k(2).set_global_batch_size(6).set_initial_model_data(init).fit(src)
    pts = [(Vectors.dense(x, y),) for x, y in [(0, 0), (0, 0.3), (0.3, 0), (9, 0), (9, 0.6), (9.6, 0)]]
    src.add_rows(pts, ["features"])
    out = model.transform(Table.from_rows(pts, ["features"]))[0]
    preds = out.column("prediction").tolist()
    assert len(set(preds[:3])) == 1 and len(set(preds[3:])) == 1 and preds[0] != preds[3]
    assert model.model_data_version() == 2  # initial model + one update


def test_random_model_data_is_java_random():
    from flink_ml_amd.utils.java import JavaRandom

    t = generate_random_kmeans_model_data(2, 3, 1.5, 42)
    cents, w = t.rows()[0]
    r = JavaRandom(42)
    assert cents[0].values.tolist() == [r.next_double() for _ in range(3)]
    assert w.values.tolist() == [1.5, 1.5]


def test_online_kmeans_decay():
    init = Table({"centroids": [[Vectors.dense(0.0, 0.0), Vectors.dense(10.0, 10.0)]],
                  "weights": [Vectors.dense(1.0, 1.0)]}, num_rows=1)
    pts = Table.from_rows([(Vectors.dense(1.0, 1.0),), (Vectors.dense(9.0, 9.0),)], ["features"])
    model = OnlineKMeans().set_k(2).set_global_batch_size(2).set_decay_factor(0.5).set_initial_model_data(init).fit(pts)
    model._stream.pull()
    cents, w = model._stream.latest()
    # weights: 1*0.5 + 1 = 1.5; lambda = 1/1.5 → c = (1-2/3)*0 + 2/3*1
    assert np.allclose(cents[0].values, [2 / 3, 2 / 3]) and np.allclose(w.values, [1.5, 1.5])


@pytest.mark.gpu
@pytest.mark.parametrize("policy,tol", [("fp64", 1e-9), ("fp32", 1e-5)])
def test_gpu_online_lr_dense_and_sparse(policy, tol):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.config import dtype_policy

    with dtype_policy(policy):
        init = Table.from_rows([(Vectors.dense(0.41233679404769874, -0.18088118293232122), 0)],
                               ["coefficient", "modelVersion"])
        src = InMemorySource()
        model = (OnlineLogisticRegression().set_reg(0.2).set_elastic_net(0.5).set_global_batch_size(10)
                 .set_initial_model_data(init).fit(src))
        pred = Table.from_rows(PREDICT, ["features", "label"])
        src.add_rows(TRAIN1, ["features", "label"])
        assert np.allclose(_raw(model.transform(pred)[0]), EXP1, atol=tol)
        src.add_rows(TRAIN2, ["features", "label"])
        assert np.allclose(_raw(model.transform(pred)[0]), EXP2, atol=tol)
        init = Table.from_rows([(Vectors.dense(*([0.01] * 10)), 0)], ["coefficient", "modelVersion"])
        src = InMemorySource()
        model = (OnlineLogisticRegression().set_reg(0.2).set_elastic_net(0.5).set_global_batch_size(9)
                 .set_initial_model_data(init).fit(src))
        src.add_rows([r[:2] for r in S1], ["features", "label"])
        assert np.allclose(_raw(model.transform(Table.from_rows(SPRED, ["features", "label"]))[0]), SEXP1, atol=tol)


@pytest.mark.gpu
def test_gpu_online_kmeans():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    test_online_kmeans_decay()
    test_online_kmeans_streaming()


def _spmd_olr_uneven(rank, world):
    """Rank 0's shard holds one more global batch than the others: every rank must stop after
    the batches ALL ranks have (the end of a stream travels in the round's payload flag)."""
    init = Table.from_rows([(Vectors.dense(0.41233679404769874, -0.18088118293232122), 0)],
                           ["coefficient", "modelVersion"])
    train = Table.from_rows(TRAIN1 + TRAIN2 + TRAIN1, ["features", "label"])
    b = 10 // world + (1 if 10 % world > rank else 0)
    off = sum(10 // world + (1 if 10 % world > r else 0) for r in range(rank))
    nb = 3 if rank == 0 else 2
    local = Table.concat([train.slice(10 * i + off, 10 * i + off + b) for i in range(nb)])
    model = (OnlineLogisticRegression().set_reg(0.2).set_elastic_net(0.5).set_global_batch_size(10)
             .set_initial_model_data(init).fit(local))
    versions = [t.rows()[0][1] for t in model.get_model_data()[0]]
    out = model.transform(Table.from_rows(PREDICT, ["features", "label"]))[0]
    return versions, _raw(out)


@pytest.mark.parametrize("world", [2, 3])
def test_online_lr_uneven_streams_stop_together(world):
    for versions, raw in run_spmd(_spmd_olr_uneven, world):
        assert versions == [1, 2]
        assert np.allclose(raw, EXP2, atol=1e-7)


def _okm_stream(rank, world, nbatches=4, seed=0):
    g = np.random.default_rng(seed)
    pts = np.concatenate([g.normal(c, 0.3, size=(60, 2)) for c in ((0, 0), (5, 5), (0, 5))])
    g.shuffle(pts)
    rows = [(Vectors.dense(*p),) for p in pts[: 12 * nbatches]]
    glob = Table.from_rows(rows, ["features"])
    b = 12 // world + (1 if 12 % world > rank else 0)
    off = sum(12 // world + (1 if 12 % world > r else 0) for r in range(rank))
    return Table.concat([glob.slice(12 * i + off, 12 * i + off + b) for i in range(nbatches)])


def _spmd_okm(rank, world):
    init = generate_random_kmeans_model_data(3, 2, 0.0, 7)
    model = (OnlineKMeans().set_k(3).set_global_batch_size(12).set_decay_factor(0.5).set_initial_model_data(init)
             .fit(_okm_stream(rank, world)))
    model._stream.drain_available()
    cents, w = model._stream.latest()
    return np.stack([c.values for c in cents]).tolist(), w.values.tolist(), model.model_data_version()


def test_online_kmeans_ranks_agree_with_one_rank():
    ref = _spmd_okm(0, 1)
    for got in run_spmd(_spmd_okm, 3):
        assert got[2] == ref[2] == 5  # initial model + 4 updates
        assert np.allclose(got[0], ref[0], atol=1e-9) and np.allclose(got[1], ref[1], atol=1e-9)


def _online_ck(rank, world, ck_dir, attempt, fail_round, which):
    import os

    os.environ["FMLX_ATTEMPT"] = str(attempt)
    from flink_ml_amd.parallel import checkpoint as ckpt

    ckpt.clear_faults()
    ckpt.enable(ck_dir, interval=2)
    if fail_round is not None:
        ckpt.inject(ckpt.FailAfter(fail_round, rank=0, on_attempt=0))
    if which == "lr":
        init = Table.from_rows([(Vectors.dense(0.41233679404769874, -0.18088118293232122), 0)],
                               ["coefficient", "modelVersion"])
        train = Table.from_rows((TRAIN1 + TRAIN2) * 3, ["features", "label"])
        b = 10 // world + (1 if 10 % world > rank else 0)
        off = sum(10 // world + (1 if 10 % world > r else 0) for r in range(rank))
        local = Table.concat([train.slice(10 * i + off, 10 * i + off + b) for i in range(6)])
        model = (OnlineLogisticRegression().set_reg(0.2).set_elastic_net(0.5).set_global_batch_size(10)
                 .set_initial_model_data(init).fit(local))
        model._stream.drain_available()
        coef, ver = model._stream.latest()
        return coef.values.tolist(), int(ver)
    init = generate_random_kmeans_model_data(3, 2, 0.0, 7)
    model = (OnlineKMeans().set_k(3).set_global_batch_size(12).set_decay_factor(0.5).set_initial_model_data(init)
             .fit(_okm_stream(rank, world, nbatches=7)))
    model._stream.drain_available()
    cents, w = model._stream.latest()
    return np.stack([c.values for c in cents]).tolist(), model.model_data_version()


@pytest.mark.parametrize("which", ["lr", "kmeans"])
def test_online_failover_resumes_exactly(which, tmp_path):
    """Online (unbounded) training checkpoints the FTRL state (z, n, coef, version) / the
    centroids and weights every 2 model versions; after an injected failure at version 5 the
    restarted job resumes from version 4, skips the consumed batches and ends identical."""
    clean = run_spmd(_online_ck, 2, str(tmp_path / "clean"), 0, None, which)
    ck = str(tmp_path / "ck")
    with pytest.raises(RuntimeError, match="injected failure"):
        run_spmd(_online_ck, 2, ck, 0, 5, which)
    resumed = run_spmd(_online_ck, 2, ck, 1, 5, which)
    for a, b in zip(clean, resumed):
        assert a[1] == b[1] and np.allclose(a[0], b[0], atol=0, rtol=0)


def _rand_sparse_rows(n, d, nnz, seed):
    g = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        idx = np.sort(g.choice(d, size=nnz, replace=False))
        lab = float(idx.sum() % 2)
        rows.append((Vectors.sparse(d, idx.tolist(), g.random(nnz).tolist()), lab, 0.5 + g.random()))
    return rows


def _train_olr(policy, rows, d, gb, weighted):
    from flink_ml_amd.config import dtype_policy

    with dtype_policy(policy):
        init = Table.from_rows([(Vectors.dense(*([0.01] * d)), 0)], ["coefficient", "modelVersion"])
        est = (OnlineLogisticRegression().set_reg(0.1).set_elastic_net(0.3).set_global_batch_size(gb)
               .set_initial_model_data(init))
        if weighted:
            est.set_weight_col("w")
        model = est.fit(Table.from_rows(rows, ["features", "label", "w"]))
        model._stream.drain_available()
        coef, ver = model._stream.latest()
        return np.asarray(coef.values), int(ver)


@pytest.mark.gpu
def test_gpu_online_lr_sparse_kernel_matches_host():
    """online.hip ftrl_grad_csr (wave per CSR row, scatter-add) + the predicated FTRL update vs
    the host implementation of the reference's sparse branch (weighted weight sums)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rows = _rand_sparse_rows(3000, 500, 17, 3)
    ref, rv = _train_olr_on("cpu", rows)
    got, gv = _train_olr("fp64", rows, 500, 600, True)
    assert gv == rv == 5
    assert np.allclose(got, ref, rtol=1e-9, atol=1e-12)


def _train_olr_on(device, rows):
    import os

    old = os.environ.get("FMLX_DEVICE")
    os.environ["FMLX_DEVICE"] = device
    from flink_ml_amd.parallel import context

    context.reset_context()
    try:
        return _train_olr("fp64", rows, 500, 600, True)
    finally:
        if old is None:
            os.environ.pop("FMLX_DEVICE", None)
        else:
            os.environ["FMLX_DEVICE"] = old
        context.reset_context()


@pytest.mark.gpu
def test_gpu_online_kmeans_device_update_matches_host():
    """Device OnlineKMeans round (assign + ordered sums, okm_local_update, okm_merge) in fp64 vs
    the host reference implementation, over several batches."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import os

    from flink_ml_amd.config import dtype_policy
    from flink_ml_amd.parallel import context

    g = np.random.default_rng(5)
    pts = np.concatenate([g.normal(c, 0.5, size=(1000, 16)) for c in range(8)])
    g.shuffle(pts)
    init = Table({"centroids": [[Vectors.dense(*p) for p in pts[:8]]], "weights": [Vectors.dense(*([1.0] * 8))]},
                 num_rows=1)
    data = Table({"features": torch.as_tensor(pts)}, num_rows=len(pts))

    def run():
        with dtype_policy("fp64"):
            m = OnlineKMeans().set_k(8).set_global_batch_size(1600).set_decay_factor(0.7).set_initial_model_data(
                init).fit(data)
            m._stream.drain_available()
            c, w = m._stream.latest()
            return np.stack([v.values for v in c]), np.asarray(w.values), m.model_data_version()

    got = run()
    os.environ["FMLX_DEVICE"] = "cpu"
    context.reset_context()
    try:
        ref = run()
    finally:
        os.environ.pop("FMLX_DEVICE", None)
        context.reset_context()
    assert got[2] == ref[2] == 6
    assert np.allclose(got[0], ref[0], rtol=1e-9, atol=1e-9) and np.allclose(got[1], ref[1], rtol=1e-12)


@pytest.mark.gpu
def test_gpu_stream_prefetch_to_device():
    """StreamTable.to_device: batches copied host→device on a side stream, handed to the consumer
    stream (record_stream) — identical values, device-resident."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    X = torch.rand(10_000, 33, dtype=torch.float64)
    t = Table({"features": X, "label": torch.arange(10_000, dtype=torch.float64)}, num_rows=10_000)
    got = list(StreamTable.from_table(t, 1000).to_device(torch.device("cuda")))
    assert len(got) == 10
    for i, b in enumerate(got):
        f = b.column("features")
        assert f.is_cuda and torch.equal(f.cpu(), X[1000 * i:1000 * (i + 1)])


def test_label_cache_tracks_base_identity_and_version():
    """FtrlTrainer._labels: slices of one resident label column share one conversion; an
    in-place change of the column, or a different column, is never served from the cache."""
    from flink_ml_amd.models.online import FtrlTrainer

    tr = FtrlTrainer(np.zeros(3), 0.1, 0.1, 0.0, 0.0, "features", "label", None)
    tr.dev = torch.device("cpu")
    tr.acc = torch.float32
    y = torch.arange(10, dtype=torch.float64)
    X = torch.zeros((10, 3))
    t = Table({"features": X, "label": y})
    a = tr._labels(t.slice(2, 5))
    assert a.dtype == torch.float32 and a.tolist() == [2.0, 3.0, 4.0]
    cached = tr._label_cache["base"][2]
    b = tr._labels(t.slice(5, 9))
    assert b.tolist() == [5.0, 6.0, 7.0, 8.0] and tr._label_cache["base"][2] is cached
    y[6] = 100.0  # in place: version bump
    assert tr._labels(t.slice(5, 9)).tolist() == [5.0, 100.0, 7.0, 8.0]
    y2 = torch.arange(10, 20, dtype=torch.float64)
    t2 = Table({"features": X, "label": y2})
    assert tr._labels(t2.slice(0, 2)).tolist() == [10.0, 11.0]


def test_model_data_stream_after_version_eviction(monkeypatch):
    """once more versions exist than the log retains, get_model_data must
    start at the oldest retained version instead of raising IndexError."""
    monkeypatch.setenv("FMLX_MODEL_VERSIONS_KEEP", "2")
    init = Table.from_rows([(Vectors.dense(0.0, 0.0), 0)], ["coefficient", "modelVersion"])
    rows = (TRAIN1 + TRAIN2) * 4  # 8 batches of 10
    model = (OnlineLogisticRegression().set_global_batch_size(10).set_initial_model_data(init)
             .fit(Table.from_rows(rows, ["features", "label"])))
    pred = Table.from_rows(PREDICT, ["features", "label"])
    model.transform(pred)  # drains the stream: versions 1..8 (only the last 2 retained)
    out = list(model.get_model_data()[0])
    versions = [int(t.rows()[0][1]) for t in out]
    assert versions == sorted(versions) and versions[-1] == 8 and len(versions) == 2
