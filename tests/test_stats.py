"""ANOVATest / FValueTest / ChiSqTest and UnivariateFeatureSelector against the reference's
expectations. Input rows and expected outputs were extracted from LIBT/stats/{ANOVATestTest,
FValueTestTest}.java and LIBT/feature/UnivariateFeatureSelectorTest.java into
tests/fixtures/stats_tests.json."""
import json
import os

import numpy as np
import pytest

from flink_ml_amd import Table, Vectors
from flink_ml_amd.models import (ANOVATest, ChiSqTest, FValueTest, UnivariateFeatureSelector,
                                 UnivariateFeatureSelectorModel)
from tests.spmd import run_spmd

FX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "stats_tests.json")))


def tab(rows):
    return Table.from_rows([(r[0], Vectors.dense(*r[1]).to_sparse() if r[2] else Vectors.dense(*r[1])) for r in rows],
                           ["label", "features"])


CHISQ_ROWS = [(0., (5, 1.)), (2., (6, 2.)), (1., (7, 2.)), (1., (5, 4.)), (0., (5, 1.)), (2., (6, 2.)), (1., (7, 2.)),
              (1., (5, 4.)), (2., (5, 1.)), (0., (5, 2.)), (0., (5, 2.)), (1., (9, 4.)), (1., (9, 3.))]
CHISQ_INT_ROWS = [(33, (5, 0)), (44, (6, 1)), (55, (7, 1)), (11, (5, 1)), (11, (5, 0)), (33, (6, 2)), (22, (7, 2)),
                  (66, (5, 3)), (77, (5, 3)), (88, (5, 4)), (77, (5, 6)), (44, (9, 6)), (11, (9, 8))]


@pytest.mark.parametrize("cls,key", [(ANOVATest, "anova"), (FValueTest, "fvalue")])
@pytest.mark.parametrize("kind", ["dense", "sparse"])
def test_anova_fvalue_flatten(cls, key, kind):
    out = cls().set_flatten(True).transform(tab(FX[key][kind + "_input"]))[0]
    assert out.column_names == ["featureIndex", "pValue", "degreeOfFreedom", "fValue"]
    got = np.array([[float(x) for x in r] for r in out.rows()])
    np.testing.assert_allclose(got, np.array(FX[key]["expected_" + kind]), atol=1e-5, equal_nan=True)


@pytest.mark.parametrize("cls,key", [(ANOVATest, "anova"), (FValueTest, "fvalue")])
def test_anova_fvalue_row(cls, key, tmp_path):
    t = cls()
    assert t.get_label_col() == "label" and t.get_features_col() == "features" and t.get_flatten() is False
    p = str(tmp_path / key)
    t.save(p)
    out = cls.load(p).transform(tab(FX[key]["dense_input"]))[0]
    assert out.column_names == ["pValues", "degreesOfFreedom", "fValues"]
    (pv, dof, fv), = out.rows()
    exp = np.array(FX[key]["expected_dense"])
    np.testing.assert_allclose(pv.values, exp[:, 1], atol=1e-5)
    assert list(dof) == [int(x) for x in exp[:, 2]]
    np.testing.assert_allclose(fv.values, exp[:, 3], atol=1e-5)


def test_chisq():
    t = Table.from_rows([(l, Vectors.dense(*f)) for l, f in CHISQ_ROWS], ["label", "features"])
    flat = ChiSqTest().set_flatten(True).transform(t)[0]
    assert flat.column_names == ["featureIndex", "pValue", "degreeOfFreedom", "statistic"]
    assert [tuple(float(x) for x in r) for r in flat.rows()] == [(0, 0.03419350755, 6, 13.61904761905),
                                                                 (1, 0.24220177737, 6, 7.94444444444)]
    (pv, dof, st), = ChiSqTest().transform(t)[0].rows()
    assert list(pv.values) == [0.03419350755, 0.24220177737] and dof == [6, 6]
    assert list(st.values) == [13.61904761905, 7.94444444444]
    ti = Table.from_rows([(l, Vectors.dense(*f)) for l, f in CHISQ_INT_ROWS], ["label", "features"])
    (pv, dof, st), = ChiSqTest().transform(ti)[0].rows()
    assert list(pv.values) == [0.35745138256, 0.39934987096] and dof == [21, 42]
    assert list(st.values) == [22.75, 43.69444444444]


def _spmd_stats(rank, world):
    t = tab(FX["anova"]["dense_input"]).partition(rank, world)
    a = [[float(x) for x in r] for r in ANOVATest().set_flatten(True).transform(t)[0].rows()]
    f = [[float(x) for x in r] for r in FValueTest().set_flatten(True).transform(
        tab(FX["fvalue"]["dense_input"]).partition(rank, world))[0].rows()]
    c = [[float(x) for x in r] for r in ChiSqTest().set_flatten(True).transform(Table.from_rows(
        [(l, Vectors.dense(*v)) for l, v in CHISQ_ROWS], ["label", "features"]).partition(rank, world))[0].rows()]
    return a, f, c


def test_stats_distributed():
    for a, f, c in run_spmd(_spmd_stats, 3):
        np.testing.assert_allclose(a, FX["anova"]["expected_dense"], atol=1e-5)
        np.testing.assert_allclose(f, FX["fvalue"]["expected_dense"], atol=1e-5)
        assert c == [[0, 0.03419350755, 6, 13.61904761905], [1, 0.24220177737, 6, 7.94444444444]]


# ------------------------------------------------------------------ UnivariateFeatureSelector
def _selectors():
    return (UnivariateFeatureSelector().set_feature_type("categorical").set_label_type("categorical"),
            UnivariateFeatureSelector().set_feature_type("continuous").set_label_type("categorical"),
            UnivariateFeatureSelector().set_feature_type("continuous").set_label_type("continuous"))


def _verify(sel, t, expected):
    out = sel.fit(t).transform(t)[0]
    for feat, o in zip(out.get_list("features"), out.get_list("output")):
        assert o.size() == len(expected)
        np.testing.assert_allclose(o.to_array(), feat.to_array()[expected], atol=1e-5)


@pytest.mark.parametrize("mode,ths,expected", [
    ("numTopFeatures", (2, 2, 2), ([0, 1], [0, 2], [0, 2])),
    ("percentile", (0.17, 0.17, 0.17), ([0], [0], [2])),
    ("fpr", (0.02, 1e-12, 0.01), ([0], [0], [2])),
    ("fdr", (0.12, 6e-12, 0.03), ([0], [0], [2])),
    ("fwe", (0.12, 6e-12, 0.03), ([0], [0], [2])),
])
def test_univariate_feature_selector_modes(mode, ths, expected):
    tables = (tab(FX["ufs"]["INPUT_CHISQ_DATA"]), tab(FX["ufs"]["INPUT_ANOVA_DATA"]),
              tab(FX["ufs"]["INPUT_FVALUE_DATA"]))
    for sel, th, t, e in zip(_selectors(), ths, tables, expected):
        _verify(sel.set_selection_mode(mode).set_selection_threshold(float(th)), t, e)


def test_univariate_feature_selector_params_and_errors(tmp_path):
    s = UnivariateFeatureSelector()
    assert s.get_features_col() == "features" and s.get_label_col() == "label" and s.get_output_col() == "output"
    assert s.get_selection_mode() == "numTopFeatures" and s.get_selection_threshold() is None
    with pytest.raises(ValueError, match="featureType's value should not be null"):
        s.get_feature_type()
    t = tab(FX["ufs"]["INPUT_ANOVA_DATA"])
    sel = UnivariateFeatureSelector().set_feature_type("continuous").set_label_type("categorical")
    with pytest.raises(ValueError, match="positive Integer"):
        sel.set_selection_threshold(50.1).fit(t)
    with pytest.raises(ValueError, match="range"):
        sel.set_selection_mode("fpr").set_selection_threshold(1.1).fit(t)
    with pytest.raises(ValueError, match="Unsupported combination"):
        UnivariateFeatureSelector().set_feature_type("categorical").set_label_type("continuous").fit(t)
    model = UnivariateFeatureSelector().set_feature_type("continuous").set_label_type("continuous") \
        .set_selection_threshold(1.0).fit(tab(FX["ufs"]["INPUT_FVALUE_DATA"]))
    with pytest.raises(ValueError, match="expecting at least 3 features"):
        model.transform(Table.from_rows([(1, Vectors.dense(1.0, 2.0))], ["label", "features"]))
    p = str(tmp_path / "ufsm")
    model.save(p)
    assert UnivariateFeatureSelectorModel.load(p).get_model_data()[0].rows()[0][0] == [2]


def test_univariate_feature_selector_model_data():
    py = tab(FX["ufs"]["PY_ANOVA_DATA"])
    sel = UnivariateFeatureSelector().set_feature_type("continuous").set_label_type("categorical") \
        .set_selection_threshold(3.0)
    model = sel.fit(py)
    assert model.get_model_data()[0].column_names == ["indices"]
    assert model.get_model_data()[0].rows()[0][0] == [0, 2, 1]
    eq = Table.from_rows([(0.0, Vectors.dense(6.0, 7.0, 0.0, 6.0, 6.0, 6.0)), (1.0, Vectors.dense(0.0, 9.0, 6.0, 0.0, 5.0, 0.0)),
                          (1.0, Vectors.dense(0.0, 9.0, 3.0, 0.0, 5.0, 0.0)), (1.0, Vectors.dense(0.0, 9.0, 8.0, 0.0, 6.0, 0.0)),
                          (2.0, Vectors.dense(8.0, 9.0, 6.0, 8.0, 4.0, 8.0)), (2.0, Vectors.dense(8.0, 9.0, 6.0, 8.0, 0.0, 8.0))],
                         ["label", "features"])
    m = UnivariateFeatureSelector().set_feature_type("categorical").set_label_type("categorical") \
        .set_selection_threshold(4.0).fit(eq)
    assert m.get_model_data()[0].rows()[0][0] == [0, 3, 5, 1]
