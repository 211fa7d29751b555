"""Out-of-core bounded fits (common/outofcore.py): the batch store's resident / cached / spilled
split reproduces the partition exactly (CPU), and on a GPU the streamed SGD trainer — resident
prefix + batches DMA'd from pinned cache memory or read from spilled files through staging —
gives the in-HBM trainer's coefficients (bit-identical with the deterministic reduction), also
through the LogisticRegression estimator with FMLX_HBM_BUDGET below the data size."""
import numpy as np
import pytest
import torch

from flink_ml_amd.common.outofcore import BatchStore, parse_bytes


def test_parse_bytes():
    assert parse_bytes("1.5G") == 3 << 29 and parse_bytes("512M") == 512 << 20 and parse_bytes("100") == 100
    assert parse_bytes("2KiB") == 2048 and parse_bytes(None) is None and parse_bytes("") is None
    with pytest.raises(ValueError):
        parse_bytes("lots")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float64])
@pytest.mark.parametrize("budget_batches,host_budget", [(0, None), (3, None), (5, 0), (100, None), (2, 3000)])
def test_batch_store_roundtrip(tmp_path, dtype, budget_batches, host_budget):
    g = torch.Generator().manual_seed(1)
    n, d, B = 1003, 7, 97
    X = torch.randn((n, d), generator=g, dtype=torch.float64).to(dtype)
    es = X.element_size()
    budget = (budget_batches + 3) * B * d * es  # + the ring's slots
    st = BatchStore(X, B, "cpu", budget, host_budget=host_budget, cache_path=str(tmp_path / "c"),
                    segment_bytes=2048)
    assert st.P == 11 and st.R == min(11, budget_batches)
    if host_budget == 0:
        assert st.stats()["cache_file_bytes"] > 0  # every cached batch spilled to files
    got = []
    for b in range(st.P):
        if st.is_resident(b):
            got.append(st.resident_view(b))
        else:
            buf = torch.empty(st.rows(b) * d * es, dtype=torch.uint8)
            st.cache.read_into(st.record(b), buf)
            got.append(buf.view(dtype).reshape(st.rows(b), d))
    assert torch.equal(torch.cat(got), X)
    st.close()


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _data(n, d, seed=0, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    X = torch.rand((n, d), generator=g, dtype=torch.float32)
    y = (X[:, : d // 2].sum(1) > d / 4).double()
    return X.to(dtype), y


@pytest.mark.gpu
@pytest.mark.parametrize("budget_batches,host_budget,det", [(0, None, True), (2, None, True), (2, 0, True),
                                                            (1, None, False), (0, 0, False)])
def test_streamed_sgd_matches_in_hbm(budget_batches, host_budget, det, monkeypatch, tmp_path):
    _need_gpu()
    from flink_ml_amd.common import outofcore
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer
    from flink_ml_amd.ops import glm as gk

    monkeypatch.setattr(gk, "DETERMINISTIC", det)
    n, d, B = 20_011, 64, 3000
    X, y = _data(n, d)
    sgd = SGD(max_iter=23, learning_rate=0.5, global_batch_size=B, tol=0.0)  # 3+ passes over 7 batches
    ref = DeviceGlmTrainer(sgd, np.zeros(d), X.cuda(), y.cuda(), None, "logistic", use_graph=False).fit()
    budget = (budget_batches + outofcore.RING_SLOTS) * B * d * 2
    tr = outofcore.StreamedGlmTrainer(sgd, np.zeros(d), X, y.cuda(), None, "logistic", torch.device("cuda"),
                                      budget, host_budget=host_budget, cache_path=str(tmp_path / "c"),
                                      segment_bytes=1 << 20)
    assert tr.store.R == budget_batches and tr.ring is not None
    if host_budget == 0:
        assert tr.store.stats()["cache_file_bytes"] > 0
    got = tr.fit()
    assert tr.rounds_executed() == 23
    assert tr.ring.h2d_bytes > 0
    tr.close()
    if det:
        np.testing.assert_array_equal(got, ref)
    else:
        np.testing.assert_allclose(got, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
def test_logistic_regression_with_hbm_budget(monkeypatch):
    _need_gpu()
    from flink_ml_amd import Table
    from flink_ml_amd.models import LogisticRegression

    X, y = _data(40_000, 32, seed=3, dtype=torch.float32)
    t = Table({"features": X, "label": y}, num_rows=40_000)
    est = LogisticRegression().set_global_batch_size(5000).set_max_iter(12).set_learning_rate(0.3)
    ref = est.fit(t).get_model_data()[0].rows()[0][0].values
    monkeypatch.setenv("FMLX_HBM_BUDGET", str(5 * 5000 * 32 * 4))  # 2 of 8 batches resident + 3 ring slots
    got = est.fit(t).get_model_data()[0].rows()[0][0].values
    np.testing.assert_allclose(got, ref, rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("budget_batches,host_budget", [(0, None), (1, 0)])
def test_streamed_kmeans_matches_in_hbm(budget_batches, host_budget, tmp_path):
    """Lloyd iterations over streamed row batches (payloads added in batch order) against the
    in-HBM loop: same counts, centroids equal to fp32 summation-order rounding."""
    _need_gpu()
    from flink_ml_amd.common import outofcore
    from flink_ml_amd.models.kmeans import kmeans_lloyd

    g = torch.Generator().manual_seed(9)
    k, D, n = 8, 64, 50_000
    centers = torch.randn((k, D), generator=g, dtype=torch.float64) * 10
    lab = torch.randint(0, k, (n,), generator=g)
    X = (centers[lab] + torch.randn((n, D), generator=g, dtype=torch.float64)).to(torch.bfloat16)
    init = X[:k].double().numpy()
    ref_c, ref_w = kmeans_lloyd(X.cuda(), init, 4, "euclidean")
    rows = 7_000
    budget = (budget_batches + outofcore.RING_SLOTS) * rows * D * 2
    got_c, got_w = outofcore.streamed_kmeans(X, init, 4, "euclidean", torch.device("cuda"), budget, batch_rows=rows,
                                             host_budget=host_budget, cache_path=str(tmp_path / "k"),
                                             segment_bytes=1 << 20)
    np.testing.assert_array_equal(got_w, ref_w)
    np.testing.assert_allclose(got_c, ref_c, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_kmeans_estimator_with_hbm_budget(monkeypatch):
    _need_gpu()
    from flink_ml_amd import Table
    from flink_ml_amd.models import KMeans

    g = torch.Generator().manual_seed(2)
    centers = torch.randn((5, 16), generator=g, dtype=torch.float64) * 8
    lab = torch.randint(0, 5, (30_000,), generator=g)
    X = (centers[lab] + torch.randn((30_000, 16), generator=g, dtype=torch.float64)).float()
    t = Table({"features": X}, num_rows=30_000)
    ref = KMeans().set_k(5).set_max_iter(5).set_seed(3).fit(t).get_model_data()[0].rows()[0]
    monkeypatch.setenv("FMLX_HBM_BUDGET", str(1_000_000))  # far below the 1.9 MB partition
    monkeypatch.setenv("FMLX_OOC_KMEANS_ROWS", "4096")
    from flink_ml_amd.common import outofcore

    monkeypatch.setattr(outofcore, "KMEANS_BATCH_ROWS", 4096)
    got = KMeans().set_k(5).set_max_iter(5).set_seed(3).fit(t).get_model_data()[0].rows()[0]
    np.testing.assert_allclose(np.stack([c.values for c in got[0]]), np.stack([c.values for c in ref[0]]),
                               rtol=1e-5, atol=1e-4)
    np.testing.assert_array_equal(got[1].values, ref[1].values)


def _csr_host(n, d, seed, max_nnz=30, dtype=torch.float32):
    from flink_ml_amd.table import SparseColumn

    g = torch.Generator().manual_seed(seed)
    counts = torch.randint(0, max_nnz + 1, (n,), generator=g)
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    indptr[1:] = torch.cumsum(counts, 0)
    idx = torch.cat([torch.sort(torch.randperm(d, generator=g)[:c]).values for c in counts.tolist()]).to(torch.int32)
    vals = torch.rand(len(idx), generator=g, dtype=torch.float64).to(dtype)
    dense = torch.zeros((n, d), dtype=torch.float64)
    dense[torch.repeat_interleave(torch.arange(n), counts), idx.long()] = vals.double()
    y = (dense @ torch.linspace(-1, 1, d, dtype=torch.float64) > 0).double()
    return SparseColumn(indptr, idx, vals, d), dense, y


@pytest.mark.parametrize("budget_batches,host_budget", [(0, None), (2, None), (3, 0), (100, None)])
def test_sparse_batch_store_roundtrip(tmp_path, budget_batches, host_budget):
    """CSR batches: the resident prefix (one rebased CSR, batches as indptr windows) and the cached
    / spilled records [indptr | indices | values] reproduce every batch exactly."""
    from flink_ml_amd.common.outofcore import SparseBatchStore

    X, _, _ = _csr_host(1003, 50, 4)
    B = 97
    probe = SparseBatchStore(X, B, "cpu", None)
    budget = 3 * probe.slot_bytes() + sum(probe.record_bytes(b) for b in range(min(budget_batches, probe.P)))
    st = SparseBatchStore(X, B, "cpu", budget, host_budget=host_budget, cache_path=str(tmp_path / "c"),
                          segment_bytes=4096)
    assert st.P == 11 and st.R == min(11, budget_batches)
    if host_budget == 0:
        assert st.stats()["cache_file_bytes"] > 0
    for b in range(st.P):
        r0 = b * B
        if st.is_resident(b):
            ip, ix, vv = st.resident_view(b)
            j0 = int(ip[0])
            ip = ip - j0
            ix, vv = ix[j0:j0 + int(ip[-1])], vv[j0:j0 + int(ip[-1])]
        else:
            buf = torch.empty(max(1, st.slot_bytes()), dtype=torch.uint8)
            st.cache.read_into(st.record(b), buf)
            ip, ix, vv = st.view(buf, b)
        want_ip = X.indptr[r0:r0 + st.rows(b) + 1] - X.indptr[r0]
        assert torch.equal(ip, want_ip)
        j0, j1 = int(X.indptr[r0]), int(X.indptr[r0 + st.rows(b)])
        assert torch.equal(ix, X.indices[j0:j1]) and torch.equal(vv, X.values[j0:j1])
    st.close()


def test_default_hbm_budget_from_free_memory(monkeypatch):
    """No FMLX_HBM_BUDGET: the budget is the device's free memory minus max(4 GiB, 10 %) (a test
    hook stands in for hipMemGetInfo), so an oversized partition streams without being asked."""
    from flink_ml_amd.common import outofcore

    monkeypatch.delenv("FMLX_HBM_BUDGET", raising=False)
    monkeypatch.setattr(outofcore, "_FREE_OVERRIDE", (100 << 30, 288 << 30))
    assert outofcore.hbm_budget() == (100 << 30) - int(0.1 * (288 << 30))
    monkeypatch.setattr(outofcore, "_FREE_OVERRIDE", (5 << 30, 8 << 30))
    assert outofcore.hbm_budget() == 1 << 30
    monkeypatch.setenv("FMLX_HBM_BUDGET", "2G")
    assert outofcore.hbm_budget() == 2 << 30


@pytest.mark.gpu
@pytest.mark.parametrize("budget_batches,host_budget", [(0, None), (2, 0)])
def test_streamed_sparse_sgd_matches_in_hbm(budget_batches, host_budget, tmp_path):
    """Bounded hinge SGD over CSR batches streamed through the ring (bucket round per batch)
    against the in-HBM sparse trainer on the same data."""
    _need_gpu()
    from flink_ml_amd.common import outofcore
    from flink_ml_amd.common.optimizer import SGD, DeviceGlmTrainer, TorchGlmTrainer

    n, d, B = 20_011, 3_000, 3_000
    X, dense, y = _csr_host(n, d, 8)
    sgd = SGD(max_iter=17, learning_rate=0.5, global_batch_size=B, tol=0.0, reg=0.01, elastic_net=0.5)
    ref = DeviceGlmTrainer(sgd, np.zeros(d), X.to("cuda"), y.cuda(), None, "hinge").fit()
    host = TorchGlmTrainer(sgd, np.zeros(d), dense, y, None, "hinge").fit()
    probe = outofcore.SparseBatchStore(X, B, "cpu", None)
    budget = outofcore.RING_SLOTS * probe.slot_bytes() + sum(probe.record_bytes(b) for b in range(budget_batches))
    tr = outofcore.StreamedGlmTrainer(sgd, np.zeros(d), X, y.cuda(), None, "hinge", torch.device("cuda"), budget,
                                      host_budget=host_budget, cache_path=str(tmp_path / "s"), segment_bytes=1 << 20)
    assert tr.sparse and tr.store.R == budget_batches and tr.ring is not None and tr.inner.bkt is not None
    got = tr.fit()
    assert tr.rounds_executed() == 17 and tr.ring.h2d_bytes > 0
    tr.close()
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(got, host, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_linear_svc_streams_sparse_by_default_budget(monkeypatch):
    """LinearSVC on a host CSR column larger than the DEFAULT budget (free memory shrunk through the
    test hook, no FMLX_HBM_BUDGET): the fit streams by itself and matches the in-HBM fit."""
    _need_gpu()
    from flink_ml_amd import Table
    from flink_ml_amd.common import optimizer, outofcore
    from flink_ml_amd.models import LinearSVC

    monkeypatch.delenv("FMLX_HBM_BUDGET", raising=False)
    X, _, y = _csr_host(30_000, 2_000, 12)
    t = Table({"features": X, "label": y}, num_rows=30_000)
    est = LinearSVC().set_global_batch_size(4000).set_max_iter(9).set_learning_rate(0.2)
    ref = est.fit(t).get_model_data()[0].rows()[0][0].values
    used = []
    real = outofcore.StreamedGlmTrainer

    class Spy(real):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            used.append(self.store.stats())

    monkeypatch.setattr(outofcore, "StreamedGlmTrainer", Spy)
    need = X.indptr.numel() * 8 + X.indices.numel() * 8
    monkeypatch.setattr(outofcore, "_FREE_OVERRIDE", (outofcore.MARGIN_MIN + need // 3, 288 << 30))
    monkeypatch.setattr(outofcore, "MARGIN_FRAC", 0.0)
    got = est.fit(t).get_model_data()[0].rows()[0][0].values
    assert used and used[0]["sparse"] and used[0]["streamed"] > 0
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
