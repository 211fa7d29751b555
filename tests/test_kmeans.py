"""KMeans / KMeansModel (reference LIBT/clustering/KMeansTest.java) on CPU incl. 4 gloo ranks,
plus GPU numerics of the MFMA assign and the deterministic centroid update."""
import numpy as np
import pytest
import torch

from flink_ml_amd import Table, Vectors
from flink_ml_amd.models import KMeans, KMeansModel
from flink_ml_amd.models.kmeans import reservoir_sample_indices
from tests.spmd import run_spmd

DATA = [Vectors.dense(0.0, 0.0), Vectors.dense(0.0, 0.3), Vectors.dense(0.3, 0.0),
        Vectors.dense(9.0, 0.0), Vectors.dense(9.0, 0.6), Vectors.dense(9.6, 0.0)]
GROUPS = [{(0.0, 0.0), (0.0, 0.3), (0.3, 0.0)}, {(9.0, 0.0), (9.0, 0.6), (9.6, 0.0)}]


def _table(rows=DATA):
    return Table.from_rows([(v,) for v in rows], ["features"])


def _groups(out):
    g = {}
    for feat, pred in out.rows():
        g.setdefault(pred, set()).add(tuple(feat.values.tolist()))
    return sorted(g.values(), key=lambda s: min(s))


def test_params():
    km = KMeans()
    assert km.get_k() == 2 and km.get_max_iter() == 20 and km.get_distance_measure() == "euclidean"
    assert km.get_init_mode() == "random" and km.get_seed() == km.get_seed()
    from flink_ml_amd.utils.java import java_string_hash

    assert km.get_seed() == java_string_hash("org.apache.flink.ml.clustering.kmeans.KMeans")
    with pytest.raises(ValueError):
        km.set_k(1)


def test_fit_predict_golden():
    model = KMeans().set_max_iter(2).set_k(2).fit(_table())
    out = model.transform(_table())[0]
    assert out.column_names == ["features", "prediction"]
    assert _groups(out) == sorted(GROUPS, key=lambda s: min(s))


@pytest.mark.parametrize("metric", ["manhattan", "cosine"])
def test_other_metrics(metric):
    rows = DATA if metric == "manhattan" else [Vectors.dense(1.0, 0.01), Vectors.dense(1.0, 0.02),
                                               Vectors.dense(0.01, 1.0), Vectors.dense(0.02, 1.0)]
    model = KMeans().set_distance_measure(metric).set_seed(7).fit(_table(rows))
    out = model.transform(_table(rows))[0]
    assert len({p for _, p in out.rows()}) == 2


def test_save_load_and_model_data(tmp_path):
    model = KMeans().set_max_iter(5).fit(_table())
    p = str(tmp_path / "km")
    model.save(p)
    loaded = KMeansModel.load(p)
    assert np.allclose(loaded.centroids(), model.centroids())
    assert _groups(loaded.transform(_table())[0]) == sorted(GROUPS, key=lambda s: min(s))
    md = loaded.get_model_data()[0].rows()[0]
    assert sorted(md[1].values.tolist()) == [3.0, 3.0]
    # byte layout: int32 k + k*(int32 2 + 2 doubles) + weights(int32 2 + 2 doubles)
    import os

    data = open(os.path.join(p, "data", "part-0-0"), "rb").read()
    assert len(data) == 4 + 2 * (4 + 16) + (4 + 16)


def test_reservoir_matches_java_random():
    from flink_ml_amd.utils.java import JavaRandom

    got = reservoir_sample_indices(500, 7, 1234)
    r = JavaRandom(1234)
    ref = list(range(7))
    for i in range(7, 500):
        j = r.next_int(i + 1)
        if j < 7:
            ref[j] = i
    assert got.tolist() == ref


def test_fewer_points_than_k():
    model = KMeans().set_k(10).fit(_table(DATA[:3]))
    assert len(model.get_model_data()[0].rows()[0][0]) == 3


def _spmd_kmeans(rank, world):
    t = _table().partition(rank, world)
    model = KMeans().set_max_iter(3).fit(t)
    return model.centroids().tolist()


def test_kmeans_four_ranks():
    res = run_spmd(_spmd_kmeans, 4)
    for r in res:
        assert np.allclose(r, res[0], equal_nan=True)
    cents = sorted(map(tuple, np.round(np.array(res[0]), 6)))
    assert np.allclose(cents, [(0.1, 0.1), (9.2, 0.2)])


def _spmd_plumbing(rank, world):
    # north-star config 1: KMeans k=2 on 100 synthetic 2-D vectors across local ranks
    g = np.random.default_rng(5)
    pts = np.concatenate([g.normal(0, 0.1, (50, 2)), g.normal(5, 0.1, (50, 2))])
    t = Table({"features": torch.as_tensor(pts)}).partition(rank, world)
    model = KMeans().set_k(2).fit(t)
    out = model.transform(t)[0]
    return sorted(map(tuple, np.round(model.centroids(), 3))), out.column("prediction").tolist(), out.column(
        "features")[:, 0].tolist()


def test_config1_plumbing_100_points_4_ranks():
    res = run_spmd(_spmd_plumbing, 4)
    assert all(r[0] == res[0][0] for r in res)
    for _, preds, xs in res:
        for p, x in zip(preds, xs):
            assert (x > 2.5) == (p == (1 if res[0][0][1][0] > 2.5 else 0))


# ------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("D", [2, 10, 64, 100, 128, 200])
@pytest.mark.parametrize("k", [2, 10, 33, 257])
def test_gpu_assign_bf16_matches_torch(D, k):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk

    g = torch.Generator().manual_seed(D * 1000 + k)
    X = torch.randn((3000, D), generator=g).to(torch.bfloat16)
    C = torch.randn((k, D), generator=g, dtype=torch.float64)
    cb = kk.CentroidBuffers(k, D, torch.device("cuda"), torch.float32)
    cb.set(C)
    lab = kk.assign(X.cuda(), cb, "euclidean").cpu().long()
    # reference on the same bf16-rounded operands, fp32 distance
    Xf, Cf = X.float(), C.to(torch.bfloat16).float()
    d = (Cf ** 2).sum(1)[None, :] - 2 * Xf @ Cf.T
    ref = torch.argmin(d, 1)
    dsel = d.gather(1, lab[:, None]).squeeze(1)
    dref = d.gather(1, ref[:, None]).squeeze(1)
    # identical except near-ties within fp32 accumulation-order noise
    assert torch.all((lab == ref) | ((dsel - dref).abs() <= 1e-3 * (1 + dref.abs())))
    assert (lab == ref).float().mean() > 0.99


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("metric", ["euclidean", "manhattan", "cosine"])
def test_gpu_assign_generic(dtype, metric):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk

    g = torch.Generator().manual_seed(1)
    X = torch.randn((2000, 37), generator=g, dtype=torch.float64)
    C = torch.randn((9, 37), generator=g, dtype=torch.float64)
    cb = kk.CentroidBuffers(9, 37, torch.device("cuda"), torch.float64 if dtype == torch.float64 else torch.float32)
    cb.set(C)
    lab = kk.assign(X.to(dtype).cuda(), cb, metric).cpu().long()
    ref = kk.torch_assign(X.to(dtype), C.to(dtype), metric)
    assert (lab == ref).float().mean() > 0.999


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["stable", "radix", "arrival"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.float64])
def test_gpu_round_payload_matches_torch(dtype, mode, monkeypatch):
    """One round's [sums | counts] against torch: the default stable counting sort and the radix
    sort are bit-reproducible, the arrival-order counting sort (k > 2048 without
    FMLX_DETERMINISTIC) reproducible to rounding (exact counts)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk
    from flink_ml_amd.ops import native

    monkeypatch.setattr(kk, "GROUP_SORT", mode != "radix")
    if mode == "arrival":  # what k > fmlx_group_stable_max_keys() takes
        monkeypatch.setattr(native.kernels(), "fmlx_group_stable_max_keys", lambda: 0)
    det = mode != "arrival"
    g = torch.Generator().manual_seed(2)
    n, D, k = 20000, 100, 10
    X = torch.rand((n, D), generator=g, dtype=torch.float64).to(dtype)
    C = X[:k].to(torch.float64)
    acc = torch.float64 if dtype == torch.float64 else torch.float32
    cb = kk.CentroidBuffers(k, D, torch.device("cuda"), acc)
    cb.set(C)
    rnd = kk.KMeansRound(X.cuda(), k, "euclidean")
    assert rnd.stable == (mode == "stable") and rnd.group == (mode == "arrival")
    p1 = rnd.run(cb).clone()
    p2 = rnd.run(cb).clone()
    if det:
        assert torch.equal(p1, p2)  # bit-reproducible
    else:
        assert torch.equal(p1[k * D:], p2[k * D:]) and torch.allclose(p1, p2, rtol=1e-6, atol=1e-4)
    lab = rnd.labels.cpu().long()
    ref_sums = torch.zeros((k, D), dtype=torch.float64).index_add_(0, lab, X.to(torch.float64))
    ref_cnt = torch.bincount(lab, minlength=k).double()
    got = p1.cpu().double()
    assert torch.allclose(got[: k * D].reshape(k, D), ref_sums, rtol=1e-5, atol=1e-3)
    assert torch.equal(got[k * D:], ref_cnt)
    rnd.finalize(cb, p1)
    assert torch.allclose(cb.cent.cpu().double(), ref_sums / ref_cnt[:, None], rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_gpu_kmeans_fit_golden():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    for dt in ("fp64", "bf16", "fp32"):
        from flink_ml_amd.config import dtype_policy

        with dtype_policy(dt):
            model = KMeans().set_max_iter(2).fit(_table())
            out = model.transform(_table())[0]
        assert _groups(out) == sorted(GROUPS, key=lambda s: min(s)), dt


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1000, 300_000])
def test_gpu_assign_fp32_euclidean_both_paths(n):
    """fp32 euclidean assign: the wave kernel (small n) and the GEMM + argmin path (large n, few
    centroids) against the fp64 torch reference; near-ties may differ only by rounding."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk

    g = torch.Generator(device="cpu").manual_seed(n)
    X = torch.rand((n, 100), generator=g)
    C = torch.rand((10, 100), generator=g)
    cb = kk.CentroidBuffers(10, 100, torch.device("cuda"), torch.float32)
    cb.set(C)
    got = kk.assign(X.cuda(), cb, "euclidean").cpu().long()
    d = torch.cdist(X.double(), C.double())
    ref = d.argmin(1)
    diff = got != ref
    if bool(diff.any()):
        gap = (d[diff, got[diff]] - d[diff, ref[diff]]).abs()
        assert float(gap.max()) < 1e-4, float(gap.max())
    assert float(diff.double().mean()) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("sched", [0, 1])
def test_gpu_assign_bf16_variants_agree(sched):
    """Both MFMA assign kernels (plain loop; pipelined with the norms in the matrix core) on
    D = 64 / 128 with a centroid count that is not a multiple of the 32-wide tile: labels equal the
    plain kernel's except at fp32 near-ties."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk

    dev = torch.device("cuda")
    try:
        for D, k in ((64, 250), (128, 97)):
            g = torch.Generator(device=dev).manual_seed(D + k)
            X = torch.rand((200_003, D), generator=g, device=dev).to(torch.bfloat16)
            C = torch.rand((k, D), generator=g, device=dev, dtype=torch.float64)
            cb = kk.CentroidBuffers(k, D, dev, torch.float32)
            cb.set(C)
            kk.set_assign_sched(0)
            ref = kk.assign(X, cb, "euclidean").long()
            kk.set_assign_sched(sched)
            lab = kk.assign(X, cb, "euclidean").long()
            assert int(lab.max()) < k and int(lab.min()) >= 0
            diff = lab != ref
            if bool(diff.any()):
                Xf, Cf = X[diff].float(), C.to(torch.bfloat16).float()
                d = (Xf ** 2).sum(1, keepdim=True) + (Cf ** 2).sum(1)[None, :] - 2.0 * Xf @ Cf.T
                g1 = d.gather(1, lab[diff][:, None]).squeeze(1)
                g0 = d.gather(1, ref[diff][:, None]).squeeze(1)
                assert bool(((g1 - g0).abs() <= 1e-4 * d.min(1).values.abs().clamp_min(1e-6)).all())
            assert float(diff.double().mean()) < 1e-3
    finally:
        kk.set_assign_sched(kk.ASSIGN_SCHED)


@pytest.mark.gpu
def test_gpu_assign_bf16_north_star_shape():
    """The MFMA assign instance the north-star shard runs (kmeans_assign_bf16_kernel<8, true>:
    D=128, k=1024) on 1.2M rows against fp32 torch distances of the same bf16 operands."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(11)
    n, D, k = 1_200_000, 128, 1024
    X = torch.rand((n, D), generator=g, device=dev).to(torch.bfloat16)
    C = torch.rand((k, D), generator=g, device=dev, dtype=torch.float64)
    cb = kk.CentroidBuffers(k, D, dev, torch.float32)
    cb.set(C)
    assert kk.mfma_ok(X, "euclidean") and cb.KS == 8
    lab = kk.assign(X, cb, "euclidean").long()
    Cf = C.to(torch.bfloat16).float()
    cn = (Cf ** 2).sum(1)
    bad = 0
    for r0 in range(0, n, 200_000):
        Xf = X[r0:r0 + 200_000].float()
        d = cn[None, :] - 2.0 * (Xf @ Cf.T)
        ref = d.argmin(1)
        got = lab[r0:r0 + 200_000]
        diff = got != ref
        if bool(diff.any()):
            dsel = d.gather(1, got[:, None]).squeeze(1)[diff]
            dref = d.gather(1, ref[:, None]).squeeze(1)[diff]
            xn = (Xf[diff] ** 2).sum(1)
            # near-ties only: within fp32 accumulation noise of the full distance ‖x‖² + d
            assert bool(((dsel - dref).abs() <= 2e-3 * (xn + dref).abs()).all())
            bad += int(diff.sum())
    assert bad / n < 2e-3


@pytest.mark.gpu
def test_gpu_round_offsets_with_empty_clusters():
    """Device cluster boundaries (sorted labels → offsets / chunk offsets, no host sync) with
    empty clusters and clusters larger than one gather chunk."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk

    g = torch.Generator().manual_seed(4)
    n, D, k = 50_000, 16, 300
    X = torch.rand((n, D), generator=g).to(torch.bfloat16)
    C = torch.cat([X[:200].double(), torch.full((100, D), 50.0, dtype=torch.float64)])  # 100 far-away centroids
    cb = kk.CentroidBuffers(k, D, torch.device("cuda"), torch.float32)
    cb.set(C)
    rnd = kk.KMeansRound(X.cuda(), k, "euclidean")
    p = rnd.run(cb).cpu().double()
    lab = rnd.labels.cpu().long()
    cnt = torch.bincount(lab, minlength=k)
    assert torch.equal(p[k * D:], cnt.double()) and int((cnt == 0).sum()) >= 100
    assert torch.equal(rnd.offsets.cpu(), torch.cat([torch.zeros(1, dtype=torch.int64), cnt.cumsum(0)]))
    ch = (cnt + kk.CHUNK - 1) // kk.CHUNK
    assert torch.equal(rnd.chunk_off.cpu(), torch.cat([torch.zeros(1, dtype=torch.int64), ch.cumsum(0)]))
    sums = torch.zeros((k, D), dtype=torch.float64).index_add_(0, lab, X.double())
    assert torch.allclose(p[: k * D].reshape(k, D), sums, rtol=1e-5, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k", [(1, 1), (1000, 7), (3_000_001, 1024), (200_000, 16384)])
def test_group_by_key_counting_sort(n, k):
    """The KMeans grouping kernel (csrc/groupsort.hip) against torch: every row once, grouped by
    key, offsets = cumulative counts, chunk offsets = cumulative ceil(count / 256); empty keys,
    one huge key (half the rows) and keys outside [0, k) (dropped)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk

    g = torch.Generator(device="cpu").manual_seed(n + k)
    keys = torch.randint(0, max(k // 2, 1), (n,), generator=g, dtype=torch.int32) * 2  # odd keys empty
    keys[: n // 2] = k - 1 if k > 1 else 0  # one huge cluster
    if n > 10:
        keys[3] = -1
        keys[5] = k  # out of range: dropped
    order, offsets, chunk_off = kk.group_by_key(keys.cuda(), k, 256)
    valid = (keys >= 0) & (keys < k)
    counts = torch.bincount(keys[valid].long(), minlength=k)
    exp_off = torch.zeros(k + 1, dtype=torch.int64)
    exp_off[1:] = torch.cumsum(counts, 0)
    assert torch.equal(offsets.cpu(), exp_off)
    exp_chk = torch.zeros(k + 1, dtype=torch.int64)
    exp_chk[1:] = torch.cumsum((counts + 255) // 256, 0)
    assert torch.equal(chunk_off.cpu(), exp_chk)
    o = order.cpu().long()
    assert torch.equal(torch.sort(o).values, torch.nonzero(valid).view(-1))  # a permutation of the valid rows
    assert torch.all(keys[o][1:] >= keys[o][:-1])  # grouped by key
    # second call reuses the re-zeroed counts (the hipGraph replay contract)
    order2, offsets2, _ = kk.group_by_key(keys.cuda(), k, 256)
    assert torch.equal(offsets2.cpu(), exp_off)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k", [(1, 1), (1000, 7), (8192, 3), (8193, 2048), (3_000_001, 1024), (700_001, 2048)])
def test_group_by_key_stable_equals_torch_stable_sort(n, k):
    """The stable counting sort (groupsort.hip st_*) equals torch's stable sort by key exactly:
    rows of a key in row order; empty keys, a huge key, keys outside [0, k) dropped, partial tiles
    and tile groups; a second call (scratch reuse) gives the same."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk

    g = torch.Generator(device="cpu").manual_seed(n * 7 + k)
    keys = torch.randint(0, max(k // 2, 1), (n,), generator=g, dtype=torch.int32) * 2
    keys[: n // 3] = k - 1 if k > 1 else 0
    if n > 10:
        keys[3] = -1
        keys[5] = k
    valid = (keys >= 0) & (keys < k)
    idx = torch.nonzero(valid).view(-1)
    ref = idx[torch.sort(keys[idx].long(), stable=True).indices]
    for _ in range(2):
        order, offsets, chunk_off = kk.group_by_key(keys.cuda(), k, 256, stable=True)
        assert torch.equal(order.cpu().long(), ref)
        counts = torch.bincount(keys[valid].long(), minlength=k)
        assert torch.equal(offsets.cpu()[1:], torch.cumsum(counts, 0)) and int(offsets[0]) == 0
        assert torch.equal(chunk_off.cpu()[1:], torch.cumsum((counts + 255) // 256, 0))


@pytest.mark.gpu
def test_gpu_round_matches_torch_and_replays():
    """One Lloyd round (assign → stable grouping → ordered gather-sums → cluster sums): equals torch
    to rounding with exact counts, is bit-reproducible run to run, and replays from a captured
    hipGraph."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from flink_ml_amd.ops import kmeans as kk
    from flink_ml_amd.utils import graphs

    g = torch.Generator().manual_seed(4)
    n, D, k = 30_011, 128, 37
    X = torch.rand((n, D), generator=g, dtype=torch.float64).to(torch.bfloat16)
    C = X[:k].to(torch.float64)
    cb = kk.CentroidBuffers(k, D, torch.device("cuda"), torch.float32)
    cb.set(C)
    rnd = kk.KMeansRound(X.cuda(), k, "euclidean")
    p1 = rnd.run(cb).clone()
    p2 = rnd.run(cb).clone()
    assert torch.equal(p1, p2)
    lab = rnd.labels.cpu().long()
    ref_sums = torch.zeros((k, D), dtype=torch.float64).index_add_(0, lab, X.to(torch.float64))
    ref_cnt = torch.bincount(lab, minlength=k).double()
    got = p1.cpu().double()
    assert torch.allclose(got[: k * D].reshape(k, D), ref_sums, rtol=1e-5, atol=1e-3)
    assert torch.equal(got[k * D:], ref_cnt)
    out = {}

    def one():
        out["p"] = rnd.run(cb)

    gr = graphs.capture(one, torch.device("cuda"))
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(out["p"], p1)
