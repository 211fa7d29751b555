"""BinaryClassificationEvaluator against the reference's expectations
(flink-ml-python/.../evaluation/tests/tests_binaryclassificationevaluator.py and
LIBT/evaluation/BinaryClassificationEvaluatorTest.java), incl. range-partitioned gloo ranks."""
import numpy as np
import pytest

from flink_ml_amd import Table, Vectors
from flink_ml_amd.models import BinaryClassificationEvaluator
from tests.spmd import run_spmd

ROWS = [(1.0, (0.1, 0.9)), (1.0, (0.2, 0.8)), (1.0, (0.3, 0.7)), (0.0, (0.25, 0.75)), (0.0, (0.4, 0.6)),
        (1.0, (0.35, 0.65)), (1.0, (0.45, 0.55)), (0.0, (0.6, 0.4)), (0.0, (0.7, 0.3)), (1.0, (0.65, 0.35)),
        (0.0, (0.8, 0.2)), (1.0, (0.9, 0.1))]
SCORE_ROWS = [(1, 0.9), (1, 0.8), (1, 0.7), (0, 0.75), (0, 0.6), (1, 0.65), (1, 0.55), (0, 0.4), (0, 0.3), (1, 0.35),
              (0, 0.2), (1, 0.1)]
MULTI = [(1.0, (0.1, 0.9)), (1.0, (0.1, 0.9)), (1.0, (0.1, 0.9)), (0.0, (0.25, 0.75)), (0.0, (0.4, 0.6)),
         (1.0, (0.1, 0.9)), (1.0, (0.1, 0.9)), (0.0, (0.6, 0.4)), (0.0, (0.7, 0.3)), (1.0, (0.1, 0.9)),
         (0.0, (0.8, 0.2)), (1.0, (0.9, 0.1))]
WEIGHTS = [0.8, 0.7, 0.5, 1.2, 1.3, 1.5, 1.4, 0.3, 0.5, 1.9, 1.2, 1.0]
EXPECTED = [0.7691481137909708, 0.3714285714285714, 0.6571428571428571]
EXPECTED_M = [0.8571428571428571, 0.9377705627705628, 0.8571428571428571, 0.6488095238095237]


def _vec(rows):
    return Table.from_rows([(l, Vectors.dense(*v)) for l, v in rows], ["label", "rawPrediction"])


def _row(out):
    return [float(x) for x in out.rows()[0]]


def test_params(tmp_path):
    e = BinaryClassificationEvaluator()
    assert e.get_label_col() == "label" and e.get_weight_col() is None and e.get_raw_prediction_col() == "rawPrediction"
    assert e.get_metrics_names() == ("areaUnderROC", "areaUnderPR")
    e.set_metrics_names("areaUnderROC").set_weight_col("weight")
    assert e.get_metrics_names() == ("areaUnderROC",)
    with pytest.raises(ValueError):
        BinaryClassificationEvaluator().set_metrics_names("accuracy")
    p = str(tmp_path / "bce")
    e.save(p)
    assert BinaryClassificationEvaluator.load(p).get_metrics_names() == ("areaUnderROC",)


def test_evaluate():
    e = BinaryClassificationEvaluator().set_metrics_names("areaUnderPR", "ks", "areaUnderROC")
    out = e.transform(_vec(ROWS))[0]
    assert out.column_names == ["areaUnderPR", "ks", "areaUnderROC"]
    np.testing.assert_allclose(_row(out), EXPECTED, atol=1e-5)
    t = Table.from_rows(SCORE_ROWS, ["label", "rawPrediction"])
    np.testing.assert_allclose(_row(e.transform(t)[0]), EXPECTED, atol=1e-5)


def test_multi_score_and_weight():
    e = BinaryClassificationEvaluator().set_metrics_names("areaUnderROC", "areaUnderPR", "ks", "areaUnderLorenz")
    np.testing.assert_allclose(_row(e.transform(_vec(MULTI))[0]), EXPECTED_M, atol=1e-5)
    tw = Table.from_rows([(l, Vectors.dense(*v), w) for (l, v), w in zip(MULTI, WEIGHTS)],
                         ["label", "rawPrediction", "weight"])
    ew = BinaryClassificationEvaluator().set_metrics_names("areaUnderROC").set_weight_col("weight")
    np.testing.assert_allclose(_row(ew.transform(tw)[0]), [0.8911680911680911], atol=1e-5)


def _spmd_eval(rank, world):
    e = BinaryClassificationEvaluator().set_metrics_names("areaUnderPR", "ks", "areaUnderROC")
    a = _row(e.transform(_vec(ROWS).partition(rank, world))[0])
    e2 = BinaryClassificationEvaluator().set_metrics_names("areaUnderROC", "areaUnderPR", "ks", "areaUnderLorenz")
    b = _row(e2.transform(_vec(MULTI).partition(rank, world))[0])
    return a, b


@pytest.mark.parametrize("world", [2, 5])
def test_evaluate_distributed(world):
    for a, b in run_spmd(_spmd_eval, world):
        np.testing.assert_allclose(a, EXPECTED, atol=1e-5)
        np.testing.assert_allclose(b, EXPECTED_M, atol=1e-5)
