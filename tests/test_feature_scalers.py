"""Scalers / VarianceThresholdSelector against the reference's published expectations
(flink-ml-python/pyflink/ml/lib/feature/tests/test_{standard,minmax,maxabs,robust}scaler.py,
test_variancethresholdselector.py and the matching Java tests)."""
import numpy as np
import pytest

from flink_ml_amd import Table, Vectors
from flink_ml_amd.models import (MaxAbsScaler, MaxAbsScalerModel, MinMaxScaler, MinMaxScalerModel, RobustScaler,
                                 RobustScalerModel, StandardScaler, StandardScalerModel, VarianceThresholdSelector,
                                 VarianceThresholdSelectorModel)
from tests.spmd import run_spmd


def vt(rows, col="input"):
    return Table.from_rows([(Vectors.dense(*r),) for r in rows], [col])


def out_vals(table, col="output"):
    return [np.asarray(v.to_array() if hasattr(v, "to_array") else v.values) for v in table.get_list(col)]


def assert_rows(actual, expected, tol=1e-6):
    assert len(actual) == len(expected)
    for a, e in zip(actual, expected):
        np.testing.assert_allclose(a, e, atol=tol, rtol=0)


SS_TRAIN = [(-2.5, 9.0, 1.0), (1.4, -5.0, 1.0), (2.0, -1.0, -2.0)]


def test_standard_scaler_params():
    s = StandardScaler()
    assert s.get_input_col() == "input" and s.get_output_col() == "output"
    assert s.get_with_mean() is False and s.get_with_std() is True
    s.set_with_mean(True).set_with_std(False)
    assert s.get_with_mean() is True and s.get_with_std() is False


@pytest.mark.parametrize("mean,std,expected", [
    (False, True, [(-1.0231819, 1.2480754, 0.5773502), (0.5729819, -0.6933752, 0.5773503),
                   (0.8185455, -0.1386750, -1.1547005)]),
    (True, False, [(-2.8, 8.0, 1.0), (1.1, -6.0, 1.0), (1.7, -2.0, -2.0)]),
    (True, True, [(-1.1459637, 1.1094004, 0.5773503), (0.45020003, -0.8320503, 0.5773503),
                  (0.69576368, -0.2773501, -1.1547005)]),
])
def test_standard_scaler_fit_predict(mean, std, expected):
    t = vt(SS_TRAIN)
    model = StandardScaler().set_with_mean(mean).set_with_std(std).fit(t)
    out = model.transform(t)[0]
    assert out.column_names == ["input", "output"]
    assert_rows(out_vals(out), expected)


def test_standard_scaler_model_data_and_save_load(tmp_path):
    t = vt(SS_TRAIN)
    model = StandardScaler().fit(t)
    md = model.get_model_data()[0]
    assert md.column_names == ["mean", "std"]
    (mean, std), = md.rows()
    np.testing.assert_allclose(mean.values, [0.3, 1.0, 0.0], atol=1e-7)
    np.testing.assert_allclose(std.values, [2.4433583, 7.2111026, 1.7320508], atol=1e-7)
    m2 = StandardScalerModel().set_model_data(md)
    assert_rows(out_vals(m2.transform(t)[0]), out_vals(model.transform(t)[0]), 1e-12)
    p = str(tmp_path / "ss")
    model.save(p)
    m3 = StandardScalerModel.load(p)
    assert_rows(out_vals(m3.transform(t)[0]), out_vals(model.transform(t)[0]), 1e-12)


MM_TRAIN = [(0.0, 3.0), (2.1, 0.0), (4.1, 5.1), (6.1, 8.1), (200.0, 400.0)]
MM_PRED = [(150.0, 90.0), (50.0, 40.0), (100.0, 50.0)]
MM_EXPECTED = [(0.75, 0.225), (0.25, 0.1), (0.5, 0.125)]


def test_min_max_scaler(tmp_path):
    s = MinMaxScaler()
    assert s.get_min() == 0.0 and s.get_max() == 1.0
    model = s.fit(vt(MM_TRAIN))
    assert_rows(out_vals(model.transform(vt(MM_PRED))[0]), MM_EXPECTED)
    (mn, mx), = model.get_model_data()[0].rows()
    np.testing.assert_allclose(mn.values, [0.0, 0.0])
    np.testing.assert_allclose(mx.values, [200.0, 400.0])
    p = str(tmp_path / "mm")
    model.save(p)
    assert_rows(out_vals(MinMaxScalerModel.load(p).transform(vt(MM_PRED))[0]), MM_EXPECTED)


def test_min_max_scaler_constant_column():
    # reference MinMaxScalerTest.testMaxValueEqualsMinValueButPredictValueNotEquals: output is 0.5*(max+min)
    train = vt([(40.0, 80.0), (40.0, 80.0), (40.0, 80.0)])
    model = MinMaxScaler().set_min(0.0).set_max(10.0).fit(train)
    out = out_vals(model.transform(vt([(30.0, 50.0)]))[0])
    assert_rows(out, [(5.0, 5.0)])


def test_max_abs_scaler(tmp_path):
    model = MaxAbsScaler().fit(vt(MM_TRAIN))
    assert_rows(out_vals(model.transform(vt(MM_PRED))[0]), MM_EXPECTED)
    (mx,), = model.get_model_data()[0].rows()
    np.testing.assert_allclose(mx.values, [200.0, 400.0])
    p = str(tmp_path / "ma")
    model.save(p)
    assert_rows(out_vals(MaxAbsScalerModel.load(p).transform(vt(MM_PRED))[0]), MM_EXPECTED)


def test_max_abs_scaler_sparse():
    train = Table.from_rows([(Vectors.sparse(4, [1, 3], [2.0, -4.0]),), (Vectors.sparse(4, [0], [-8.0]),)],
                            ["input"])
    model = MaxAbsScaler().fit(train)
    out = model.transform(train)[0].get_list("output")
    assert out[0].size() == 4 and list(out[0].indices) == [1, 3]
    np.testing.assert_allclose(out[0].to_array(), [0, 1.0, 0, -1.0])
    np.testing.assert_allclose(out[1].to_array(), [-1.0, 0, 0, 0])


RS_TRAIN = [(float(i), -float(i)) for i in range(9)]


def test_robust_scaler(tmp_path):
    s = RobustScaler()
    assert (s.get_lower(), s.get_upper(), s.get_relative_error()) == (0.25, 0.75, 0.001)
    assert s.get_with_centering() is False and s.get_with_scaling() is True
    model = s.fit(vt(RS_TRAIN))
    pred = vt([(3.0, -3.0), (6.0, -6.0), (99.0, -99.0)])
    expected = [(0.75, -0.75), (1.5, -1.5), (24.75, -24.75)]
    assert_rows(out_vals(model.transform(pred)[0]), expected)
    (med, rng), = model.get_model_data()[0].rows()
    np.testing.assert_allclose(med.values, [4.0, -4.0])
    np.testing.assert_allclose(rng.values, [4.0, 4.0])
    centered = RobustScaler().set_with_centering(True).fit(vt(RS_TRAIN)).transform(pred)[0]
    assert_rows(out_vals(centered), [(-0.25, 0.25), (0.5, -0.5), (23.75, -23.75)])
    p = str(tmp_path / "rs")
    model.save(p)
    assert_rows(out_vals(RobustScalerModel.load(p).transform(pred)[0]), expected)


VT_TRAIN = [(5.0, 7.0, 0.0, 7.0, 6.0, 0.0), (0.0, 9.0, 6.0, 0.0, 5.0, 9.0), (0.0, 9.0, 3.0, 0.0, 5.0, 5.0),
            (1.0, 9.0, 8.0, 5.0, 7.0, 4.0), (9.0, 8.0, 6.0, 5.0, 4.0, 4.0), (6.0, 9.0, 7.0, 0.0, 2.0, 0.0)]


def test_variance_threshold_selector(tmp_path):
    s = VarianceThresholdSelector()
    assert s.get_variance_threshold() == 0.0
    model = s.set_variance_threshold(8.0).fit(vt(VT_TRAIN))
    pred = vt([(1.0, 2.0, 3.0, 4.0, 5.0, 6.0), (0.1, 0.2, 0.3, 0.4, 0.5, 0.6)])
    assert_rows(out_vals(model.transform(pred)[0]), [(1.0, 4.0, 6.0), (0.1, 0.4, 0.6)])
    (nf, idx), = model.get_model_data()[0].rows()
    assert nf == 6 and list(idx) == [0, 3, 5]
    with pytest.raises(Exception, match="but VarianceThresholdSelector is expecting"):
        model.transform(vt([(1.0, 2.0, 3.0)]))
    p = str(tmp_path / "vts")
    model.save(p)
    m2 = VarianceThresholdSelectorModel.load(p)
    assert_rows(out_vals(m2.transform(pred)[0]), [(1.0, 4.0, 6.0), (0.1, 0.4, 0.6)])


def _spmd_scalers(rank, world):
    from flink_ml_amd.parallel.context import get_context

    t = vt(SS_TRAIN).partition(get_context().rank, get_context().world_size)
    model = StandardScaler().set_with_mean(True).fit(t)
    (mean, std), = model.get_model_data()[0].rows()
    rs = RobustScaler().fit(vt(RS_TRAIN).partition(rank, world))
    (med, rng), = rs.get_model_data()[0].rows()
    return mean.values.tolist(), std.values.tolist(), med.values.tolist(), rng.values.tolist()


def test_scalers_distributed():
    res = run_spmd(_spmd_scalers, 2)
    for mean, std, med, rng in res:
        np.testing.assert_allclose(mean, [0.3, 1.0, 0.0], atol=1e-7)
        np.testing.assert_allclose(std, [2.4433583, 7.2111026, 1.7320508], atol=1e-7)
        np.testing.assert_allclose(med, [4.0, -4.0])
        np.testing.assert_allclose(rng, [4.0, 4.0])
