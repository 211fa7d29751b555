"""KNN predict on the GPU: the fused distance + top-k kernel (``ops/csrc/knn.hip``) against a
plain PyTorch fp64 reference of the same op, and KnnModel end to end against the CPU path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _ref_topk(G, qn, tn, k):
    # same fp32 distance expression, ranked in fp64 with a stable sort (ties → lower index)
    d = torch.sqrt(torch.abs((qn[:, None] + tn[None, :]) - 2.0 * G)).double().cpu()
    return torch.sort(d, dim=1, stable=True).indices[:, :k], torch.sort(d, dim=1, stable=True).values[:, :k]


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8, 13, 16, 32])
@pytest.mark.parametrize("n", [37, 1000, 4099, 20000])
def test_topk_kernel_matches_torch(k, n):
    from flink_ml_amd.ops import knn as ko

    if k > n:
        pytest.skip("k > n")
    g = torch.Generator(device="cpu").manual_seed(k * 7919 + n)
    d = 24
    Q = torch.randn((301, d), generator=g).cuda()
    T = torch.randn((n, d), generator=g).cuda()
    G = Q @ T.t()
    qn, tn = (Q * Q).sum(1), (T * T).sum(1)
    idx, dist = ko.topk_from_products(G, qn, tn, k, with_dist=True)
    ridx, rdist = _ref_topk(G, qn, tn, k)
    torch.testing.assert_close(dist.double().cpu(), rdist, rtol=2e-7, atol=0)
    # same distances; indices equal wherever the distance is not tied with a neighbour
    assert (idx.long().cpu() == ridx).float().mean() > 0.999


def test_topk_ties_go_to_lower_index():
    from flink_ml_amd.ops import knn as ko

    g = torch.Generator(device="cpu").manual_seed(3)
    base = torch.randn((50, 8), generator=g)
    T = torch.cat([base, base, base]).cuda()          # every point three times: exact ties
    Q = torch.randn((64, 8), generator=g).cuda()
    G = Q @ T.t()
    idx = ko.topk_from_products(G, (Q * Q).sum(1), (T * T).sum(1), 6).long().cpu()
    ridx, _ = _ref_topk(G, (Q * Q).sum(1), (T * T).sum(1), 6)
    assert torch.equal(idx, ridx)
    # each duplicated pair appears in index order
    assert torch.all(idx[:, 0] < idx[:, 1]) and torch.all(idx[:, 0] % 50 == idx[:, 1] % 50)


def test_topk_misaligned_rows_and_nan():
    from flink_ml_amd.ops import knn as ko

    g = torch.Generator(device="cpu").manual_seed(5)
    n = 1001                                            # odd n → scalar path
    Q = torch.randn((40, 5), generator=g).cuda()
    T = torch.randn((n, 5), generator=g).cuda()
    G = Q @ T.t()
    tn = (T * T).sum(1)
    tn[7] = float("nan")                                # a NaN distance ranks last
    idx, dist = ko.topk_from_products(G, (Q * Q).sum(1), tn, 4, with_dist=True)
    assert not torch.any(idx == 7)
    ridx, rdist = _ref_topk(G, (Q * Q).sum(1), tn.nan_to_num(float("inf")), 4)
    torch.testing.assert_close(dist.double().cpu(), rdist, rtol=2e-7, atol=0)


def test_knn_model_gpu_matches_cpu():
    from flink_ml_amd import Table
    from flink_ml_amd.models import Knn

    rng = np.random.default_rng(0)
    centers = rng.normal(size=(4, 16)) * 4
    lab = rng.integers(0, 4, 3000)
    X = centers[lab] + rng.normal(size=(3000, 16))
    Xq = centers[lab[:500]] + rng.normal(size=(500, 16))
    train = Table({"features": torch.tensor(X, dtype=torch.float32).cuda(),
                   "label": torch.tensor(lab, dtype=torch.float64).cuda()})
    model = Knn().set_k(7).fit(train)
    pred = model.transform(Table({"features": torch.tensor(Xq, dtype=torch.float32).cuda()}))[0]
    p_gpu = pred.column("prediction").cpu().numpy()
    # fp64 host reference of the same predictor
    d = np.sqrt(np.abs((Xq ** 2).sum(1)[:, None] + (X ** 2).sum(1)[None, :] - 2 * Xq @ X.T))
    nn = np.argsort(d, axis=1, kind="stable")[:, :7]
    votes = np.array([np.bincount(lab[r], minlength=4).argmax() for r in nn])
    assert (p_gpu == votes).mean() > 0.99


@pytest.mark.parametrize("nq,n,k", [(3, 50000, 5), (700, 9000, 32), (64, 200003, 7)])
def test_topk_segmented_merge(nq, n, k):
    from flink_ml_amd.ops import knn as ko

    assert ko.segments(nq, n) > 1 or n < 2 * ko.MIN_SEGMENT
    g = torch.Generator(device="cpu").manual_seed(nq + n)
    Q = torch.randn((nq, 6), generator=g).cuda()
    T = torch.randn((n, 6), generator=g).cuda()
    G = Q @ T.t()
    qn, tn = (Q * Q).sum(1), (T * T).sum(1)
    idx, dist = ko.topk_from_products(G, qn, tn, k, with_dist=True)
    ridx, rdist = _ref_topk(G, qn, tn, k)
    torch.testing.assert_close(dist.double().cpu(), rdist, rtol=2e-7, atol=0)
    assert (idx.long().cpu() == ridx).float().mean() > 0.999


# ---- fused distance + top-k kernel (one kernel, fp32 matrix cores, no nq×n block in HBM)

def _int_data(nq, n, d, seed, lo=-3, hi=4):
    # small integers: every product, norm and distance is exact in fp32, so the fused kernel's
    # ranking must equal the fp64 ranking exactly, ties (there are many) going to the lower index
    g = torch.Generator(device="cpu").manual_seed(seed)
    Q = torch.randint(lo, hi, (nq, d), generator=g).double()
    T = torch.randint(lo, hi, (n, d), generator=g).double()
    return Q, T


def _ref_fp64(Q, T, k):
    d2 = ((Q * Q).sum(1)[:, None] + (T * T).sum(1)[None, :] - 2.0 * Q @ T.t()).abs().sqrt()
    s = torch.sort(d2, dim=1, stable=True)
    return s.indices[:, :k], s.values[:, :k]


@pytest.mark.parametrize("d", [1, 3, 8, 24, 100, 128])
@pytest.mark.parametrize("k", [1, 3, 5, 16, 33, 64])
def test_fused_topk_exact_vs_fp64(d, k):
    from flink_ml_amd.ops import knn as ko

    n = 4099
    Q, T = _int_data(301, n, d, seed=d * 101 + k)
    pack = ko.TrainPack(T.float().cuda(), (T * T).sum(1).cuda())
    idx, dist = ko.fused_topk(Q.float().cuda(), pack, k, with_dist=True)
    ridx, rdist = _ref_fp64(Q, T, k)
    assert torch.equal(idx.long().cpu(), ridx)
    torch.testing.assert_close(dist.double().cpu(), rdist, rtol=1e-6, atol=0)


@pytest.mark.parametrize("segments", [1, 2, 5, 64])
@pytest.mark.parametrize("n", [37, 64, 1000, 20011])
def test_fused_topk_segments_and_tails(segments, n):
    from flink_ml_amd.ops import knn as ko

    k = min(9, n)
    Q, T = _int_data(130, n, 17, seed=n + segments)
    pack = ko.TrainPack(T.float().cuda(), (T * T).sum(1).cuda())
    idx = ko.fused_topk(Q.float().cuda(), pack, k, segments=segments)
    ridx, _ = _ref_fp64(Q, T, k)
    assert torch.equal(idx.long().cpu(), ridx)


def test_fused_topk_random_floats_and_nan():
    from flink_ml_amd.ops import knn as ko

    g = torch.Generator(device="cpu").manual_seed(11)
    Q = torch.randn((1000, 64), generator=g)
    T = torch.randn((30000, 64), generator=g)
    tn = (T * T).sum(1)
    tn[5] = float("nan")                                 # a NaN distance ranks last: never chosen
    pack = ko.TrainPack(T.cuda(), tn.cuda())
    idx, dist = ko.fused_topk(Q.cuda(), pack, 20, with_dist=True)
    assert not torch.any(idx == 5)
    tn_ref = tn.double().clone()
    tn_ref[5] = float("inf")
    d2 = ((Q.double() ** 2).sum(1)[:, None] + tn_ref[None, :] - 2.0 * Q.double() @ T.double().t()).abs().sqrt()
    rd, ri = torch.sort(d2, dim=1, stable=True)
    torch.testing.assert_close(dist.double().cpu(), rd[:, :20], rtol=1e-5, atol=1e-5)
    assert (idx.long().cpu() == ri[:, :20]).float().mean() > 0.999


def test_knn_model_routes_fused_for_k64():
    from flink_ml_amd import Table
    from flink_ml_amd.models import Knn

    Q, T = _int_data(257, 5000, 12, seed=2)
    lab = (T[:, 0] > 0).double() + (T[:, 1] > 0).double()
    model = Knn().set_k(64).fit(Table({"features": T.float().cuda(), "label": lab.cuda()}))
    pred = model.transform(Table({"features": Q.float().cuda()}))[0].column("prediction").cpu()
    ridx, _ = _ref_fp64(Q, T, 64)
    from flink_ml_amd.models.knn import knn_vote

    ref = knn_vote(lab[ridx], torch.unique(lab))
    assert torch.equal(pred.double(), ref.double())



# ---- any k, fp32 / fp64: radix selection over the product block (ops/csrc/knn_select.hip)

@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("k", [1, 65, 300, 1000, 4099])
def test_select_topk_exact_vs_fp64(dtype, k):
    """Integer data: every distance is exact, so the ranking must equal the fp64 stable sort
    exactly — the many ties going to the lower index (KnnModel.java:154-194), k beyond the
    fused kernel's 64 up to the whole training set."""
    from flink_ml_amd.ops import knn as ko

    n = 4099
    Q, T = _int_data(97, n, 11, seed=k + (7 if dtype == torch.float64 else 0))
    q, t = Q.to(dtype).cuda(), T.to(dtype).cuda()
    idx = ko.select_topk(q @ t.t(), (q * q).sum(1), (t * t).sum(1), k)
    ridx, _ = _ref_fp64(Q, T, k)
    assert torch.equal(idx.long().cpu(), ridx)


def test_select_topk_fp64_random_and_nan():
    from flink_ml_amd.ops import knn as ko

    g = torch.Generator(device="cpu").manual_seed(13)
    Q = torch.randn((200, 40), generator=g, dtype=torch.float64)
    T = torch.randn((50000, 40), generator=g, dtype=torch.float64)
    tn = (T * T).sum(1)
    tn[9] = float("nan")                                 # a NaN distance ranks last: never chosen
    G = Q.cuda() @ T.cuda().t()
    idx = ko.select_topk(G, (Q * Q).sum(1).cuda(), tn.cuda(), 777)
    assert not torch.any(idx == 9)
    tn_ref = tn.clone()
    tn_ref[9] = float("inf")
    d2 = ((Q * Q).sum(1)[:, None] + tn_ref[None, :] - 2.0 * G.cpu()).abs()
    ri = torch.sort(d2, dim=1, stable=True).indices[:, :777]
    assert torch.equal(idx.long().cpu(), ri)


@pytest.mark.parametrize("policy,k", [("fp32", 100), ("fp64", 100), ("fp64", 5)])
def test_knn_model_large_k_and_fp64_on_select_kernel(policy, k, monkeypatch):
    """KnnModel beyond the fused kernel's k and in the fp64 parity mode runs the select kernel (no
    torch top-k) and equals the fp64 reference vote."""
    from flink_ml_amd import Table
    from flink_ml_amd.config import dtype_policy
    from flink_ml_amd.models import Knn
    from flink_ml_amd.models.knn import knn_vote
    from flink_ml_amd.ops import knn as ko

    def no_topk(*a, **kw):
        raise AssertionError("torch.topk on the KNN GPU path")

    monkeypatch.setattr(torch, "topk", no_topk)
    called = []
    real = ko.select_topk
    monkeypatch.setattr(ko, "select_topk", lambda *a: called.append(1) or real(*a))
    Q, T = _int_data(301, 6000, 150, seed=k)  # D 150 > the fused kernel's 128
    lab = (T[:, 0] > 0).double() + (T[:, 1] > 0).double()
    with dtype_policy(policy):
        model = Knn().set_k(k).fit(Table({"features": T.cuda(), "label": lab.cuda()}))
        pred = model.transform(Table({"features": Q.cuda()}))[0].column("prediction").cpu()
    assert called
    ridx, _ = _ref_fp64(Q, T, k)
    ref = knn_vote(lab[ridx], torch.unique(lab))
    assert torch.equal(pred.double(), ref.double())


@pytest.mark.parametrize("k", [1, 300, 2000])
def test_select_topk_fp32_continuous_fast_path(k):
    """Continuous fp32 data: the select kernel's collect-and-sort path (the k-th key's bin and all
    below fit the LDS after a radix pass) must give exactly the stable sort of the same keys."""
    from flink_ml_amd.ops import knn as ko

    g = torch.Generator(device="cpu").manual_seed(k + 17)
    Q = torch.randn((64, 24), generator=g)
    T = torch.randn((20000, 24), generator=g)
    G = Q.cuda() @ T.cuda().t()
    qn, tn = (Q * Q).sum(1), (T * T).sum(1)
    idx = ko.select_topk(G, qn.cuda(), tn.cuda(), k)
    d2 = ((qn[:, None] + tn[None, :]) - 2.0 * G.cpu()).abs()
    ri = torch.sort(d2, dim=1, stable=True).indices[:, :k]
    assert torch.equal(idx.long().cpu(), ri)
