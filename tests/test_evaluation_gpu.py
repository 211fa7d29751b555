"""K21 on the device (ops/csrc/binclass.hip + the radix.hip 64-bit sort): the reference's
evaluator goldens on cuda, and random / tie-heavy / NaN / weighted inputs against the fp64 torch
reference of the same metrics (models/evaluation.py's CPU path), across many 4096-row tiles so
that tie groups straddle tile boundaries."""
import numpy as np
import pytest
import torch

from flink_ml_amd.models import BinaryClassificationEvaluator
from flink_ml_amd.models.evaluation import compute_metrics
from tests.test_evaluation import EXPECTED, EXPECTED_M, MULTI, ROWS, WEIGHTS, _row, _vec

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_goldens_on_device():
    _need_gpu()
    from flink_ml_amd import Table, Vectors

    e = BinaryClassificationEvaluator().set_metrics_names("areaUnderPR", "ks", "areaUnderROC")
    np.testing.assert_allclose(_row(e.transform(_vec(ROWS))[0]), EXPECTED, atol=1e-9)
    e2 = BinaryClassificationEvaluator().set_metrics_names("areaUnderROC", "areaUnderPR", "ks", "areaUnderLorenz")
    np.testing.assert_allclose(_row(e2.transform(_vec(MULTI))[0]), EXPECTED_M, atol=1e-9)
    tw = Table.from_rows([(l, Vectors.dense(*v), w) for (l, v), w in zip(MULTI, WEIGHTS)],
                         ["label", "rawPrediction", "weight"])
    ew = BinaryClassificationEvaluator().set_metrics_names("areaUnderROC").set_weight_col("weight")
    np.testing.assert_allclose(_row(ew.transform(tw)[0]), [0.8911680911680911], atol=1e-9)


@pytest.mark.parametrize("n,kind,weighted", [
    (1, "rand", False), (7, "rand", True), (4096, "ties", False), (4097, "rand", False),
    (50_000, "ties", True), (123_457, "rand", True), (200_000, "nan", False), (60_000, "zeros", False),
    (30_000, "const", True), (300_000, "ties_wide", False)])
def test_device_metrics_match_torch(n, kind, weighted):
    _need_gpu()
    g = torch.Generator().manual_seed(n)
    s = torch.rand(n, generator=g, dtype=torch.float64)
    if kind == "ties":
        s = torch.round(s * 20) / 20  # 21 distinct scores: groups of ~n/20 rows over many tiles
    elif kind == "ties_wide":
        s = torch.round(s * 3) / 3
    elif kind == "nan":
        s[torch.rand(n, generator=g) < 0.05] = float("nan")
        s[torch.rand(n, generator=g) < 0.05] = float("inf")
    elif kind == "zeros":
        s = torch.where(torch.rand(n, generator=g) < 0.5, torch.zeros_like(s), -torch.zeros_like(s))
        s[: n // 3] = torch.rand(n // 3, generator=g, dtype=torch.float64)
    elif kind == "const":
        s = torch.full((n,), 0.5, dtype=torch.float64)
    p = torch.rand(n, generator=g) < 0.4
    w = torch.rand(n, generator=g, dtype=torch.float64) + 0.5 if weighted else torch.ones(n, dtype=torch.float64)
    ref = compute_metrics(s, p, w)
    got = compute_metrics(s.cuda(), p.cuda(), w.cuda())
    for k in ref:
        r, v = ref[k], got[k]
        if np.isnan(r):
            assert np.isnan(v), k
        else:
            assert abs(v - r) <= 1e-9 * max(1.0, abs(r)), (k, v, r)


def test_sort_u64_stable_and_segmented():
    """fmlx_sort_u64: stable within equal keys, segments never mix, any bit range."""
    _need_gpu()
    from flink_ml_amd.ops import sorting

    g = torch.Generator().manual_seed(3)
    n = 70_001
    keys = torch.randint(0, 1 << 40, (n,), generator=g, dtype=torch.int64) << 8
    keys[: n // 2] = keys[: n // 2] % 977 << 8  # many duplicates in the first segment
    vals = torch.arange(n, dtype=torch.int32)
    bounds = [0, 12_345, 12_345, 50_000, n]
    ks, vs = sorting.sort_u64(keys.cuda(), vals.cuda(), bounds, 8, 48)
    ks, vs = ks.cpu(), vs.cpu()
    for a, b in zip(bounds[:-1], bounds[1:]):
        seg_k = keys[a:b].numpy().astype(np.uint64)
        order = np.argsort(seg_k, kind="stable")
        np.testing.assert_array_equal(vs[a:b].numpy(), vals[a:b].numpy()[order])
        np.testing.assert_array_equal(ks[a:b].numpy().astype(np.uint64), seg_k[order])
