"""K22 / K20 on the device (ops/csrc/catstats.hip + the radix.hip 64-bit sort): distinct values,
label counts and (feature, value, label) contingency tables against numpy, and NaiveBayes /
ChiSqTest / ANOVATest fitted on cuda against the same stages on the CPU reference path — integer
(categorical, the reference benchmarks' shape) and general (non-integer, NaN, −0) values."""
import contextlib

import numpy as np
import pytest
import torch

from flink_ml_amd import Table
from flink_ml_amd.parallel import context as pctx

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@contextlib.contextmanager
def on_cpu():
    old = pctx._CTX
    pctx.set_context(pctx.SPMDContext(device=torch.device("cpu")))
    try:
        yield
    finally:
        pctx.set_context(old)


def test_sorted_unique_and_counts():
    _need_gpu()
    from flink_ml_amd.ops import catstats

    g = torch.Generator().manual_seed(0)
    ints = torch.randint(-7, 40, (100_003,), generator=g).double()
    np.testing.assert_array_equal(catstats.sorted_unique(ints.cuda()).cpu().numpy(), np.unique(ints.numpy()))
    fl = torch.round(torch.randn(70_000, generator=g, dtype=torch.float64) * 100) / 7
    fl[::11] = -0.0
    fl[5::13] = 0.0
    got = catstats.sorted_unique(fl.cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, np.unique(fl.numpy()))
    li = torch.randint(0, 13, (50_000,), generator=g)
    np.testing.assert_array_equal(catstats.label_counts(li.cuda(), 13).cpu().numpy(),
                                  np.bincount(li.numpy(), minlength=13))
    assert catstats.flags(torch.tensor([[1.0, 2.0], [3.0, float("nan")]]).cuda())[2]
    assert catstats.flags(torch.tensor([[1.0, float("inf")]]).cuda())[2]
    assert catstats.flags(torch.tensor([[-4.0, 7.0]]).cuda()) == (-4.0, 7.0, False)


@pytest.mark.parametrize("kind", ["int", "int_wide", "float", "float_many"])
def test_value_label_counts_match_numpy(kind):
    _need_gpu()
    from flink_ml_amd.ops import catstats

    g = torch.Generator().manual_seed(5)
    n, d, L = 40_000, 37, 6
    if kind == "int":
        X = torch.randint(0, 20, (n, d), generator=g).double()
    elif kind == "int_wide":
        X = torch.randint(-3, 900, (n, d), generator=g).double()  # table beyond LDS: global atomics
    elif kind == "float":
        X = torch.round(torch.rand((n, d), generator=g, dtype=torch.float64) * 30) / 4 + 0.1
        X[::17, 3] = float("nan")
    else:
        X = torch.rand((n, d), generator=g, dtype=torch.float64)  # nearly every value distinct
    li = torch.randint(0, L, (n,), generator=g)
    counts, vals, slots = catstats.value_label_counts(X.cuda(), li.cuda(), L)
    for j in range(d):
        col = X[:, j].numpy()
        u = np.unique(col)
        if np.isnan(u).any():  # np.unique keeps one NaN per NaN; the device folds them into one
            u = np.concatenate([u[~np.isnan(u)], [np.nan]])
        np.testing.assert_array_equal(vals[j], u)
        codes = np.searchsorted(u[~np.isnan(u)], col)
        codes[np.isnan(col)] = len(u) - 1
        ref = np.zeros((L, len(u)), dtype=np.int64)
        np.add.at(ref, (li.numpy(), codes), 1)
        np.testing.assert_array_equal(counts[j][:, slots[j]], ref)


def _nb_table(kind, n=20_000, d=12):
    g = torch.Generator().manual_seed(11)
    X = torch.randint(0, 20, (n, d), generator=g).double()
    if kind == "float":
        X = X / 8 - 0.75  # exact in fp32 (the device compute dtype)
    y = torch.randint(0, 10, (n,), generator=g).double() * 2 + 1
    return Table({"features": X, "label": y}, num_rows=n)


@pytest.mark.parametrize("kind", ["int", "float"])
def test_naive_bayes_device_matches_cpu(kind):
    _need_gpu()
    from flink_ml_amd.models import NaiveBayes

    t = _nb_table(kind)
    dev = NaiveBayes().set_smoothing(0.5).fit(t).get_model_data()[0].rows()[0]
    with on_cpu():
        ref = NaiveBayes().set_smoothing(0.5).fit(t).get_model_data()[0].rows()[0]
    for ra, rb in zip(dev[0], ref[0]):
        for ma, mb in zip(ra, rb):
            assert list(ma) == list(mb)
            np.testing.assert_allclose(list(ma.values()), list(mb.values()), rtol=1e-12)
    np.testing.assert_allclose(dev[1].values, ref[1].values, rtol=1e-12)
    assert list(dev[2].values) == list(ref[2].values)


@pytest.mark.parametrize("kind", ["int", "float"])
def test_chisq_and_anova_device_match_cpu(kind):
    _need_gpu()
    from flink_ml_amd.models import ANOVATest, ChiSqTest

    t = _nb_table(kind, n=5_000, d=6)
    got = [[float(x) for x in r] for r in ChiSqTest().set_flatten(True).transform(t)[0].rows()]
    an = [[float(x) for x in r] for r in ANOVATest().set_flatten(True).transform(t)[0].rows()]
    with on_cpu():
        ref = [[float(x) for x in r] for r in ChiSqTest().set_flatten(True).transform(t)[0].rows()]
        anr = [[float(x) for x in r] for r in ANOVATest().set_flatten(True).transform(t)[0].rows()]
    assert got == ref
    np.testing.assert_allclose(np.array(an), np.array(anr), rtol=1e-9)


def _shard_table(kind, rank, world):
    t = _nb_table(kind, n=6_000, d=5)
    X, y = t.column("features").clone(), t.column("label")
    if kind == "float":
        X[4000:, 2] = 9.375  # a value only the last rank's rows hold (the union must add it)
        X[:50, 3] = -0.0
    cut = [0, 3_500, 6_000] if world == 2 else [0, 6_000]
    s, e = cut[rank], cut[rank + 1]
    return Table({"features": X[s:e], "label": y[s:e]}, num_rows=e - s)


def _dist_stats_worker(rank, world, kind):
    from flink_ml_amd.models import ChiSqTest, NaiveBayes
    from flink_ml_amd.models import naive_bayes, stats

    def keyed_shuffle(*a, **k):  # the torch.unique / argsort keyed-shuffle path must not run on GPUs
        raise AssertionError("library-op keyed shuffle on a GPU rank")

    stats.value_label_counts = naive_bayes.value_label_counts = keyed_shuffle
    t = _shard_table(kind, rank, world)
    chi = [[float(v) for v in r] for r in ChiSqTest().set_flatten(True).transform(t)[0].rows()]
    nb = NaiveBayes().set_smoothing(0.5).fit(t).get_model_data()[0].rows()[0]
    theta = [[sorted(m.items()) for m in row] for row in nb[0]]
    return chi, theta, list(nb[1].values), list(nb[2].values)


@pytest.mark.parametrize("kind", ["int", "float"])
def test_chisq_and_naive_bayes_two_ranks_match_one(kind):
    """ChiSqTest / NaiveBayes across ranks on the native contingency kernels — the
    integer table all-reduced, or (general values) the union of the ranks' sorted distinct lists
    — equal the one-rank result on the whole data."""
    _need_gpu()
    from tests.spmd import run_spmd

    env = {"FMLX_DEVICE": "cuda:0", "FMLX_XGMI": "0"}
    res = run_spmd(_dist_stats_worker, 2, kind, env=env, timeout=300)
    (one,) = run_spmd(_dist_stats_worker, 1, kind, env=env, timeout=300)
    for r in res:
        assert r[0] == one[0]
        assert r[1] == one[1] and r[3] == one[3]
        np.testing.assert_allclose(r[2], one[2], rtol=1e-12)
