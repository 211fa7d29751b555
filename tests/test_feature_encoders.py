"""Encoders against the reference's expectations (flink-ml-python/.../feature/tests/
test_{onehotencoder,stringindexer,indextostringmodel,vectorindexer,kbinsdiscretizer,imputer}.py,
LIBT/feature/stringindexer/StringIndexerTest.java, KBinsDiscretizerTest.java)."""
import math

import numpy as np
import pytest

from flink_ml_amd import Table, Vectors
from flink_ml_amd.io import read_write as rw
from flink_ml_amd.models import (Imputer, ImputerModel, IndexToStringModel, KBinsDiscretizer, KBinsDiscretizerModel,
                                 OneHotEncoder, OneHotEncoderModel, StringIndexer, StringIndexerModel, VectorIndexer,
                                 VectorIndexerModel)
from flink_ml_amd.utils.java import java_number_to_string
from tests.spmd import run_spmd


def arr(v):
    return np.asarray(v.to_array()) if hasattr(v, "to_array") else np.asarray(v)


# ------------------------------------------------------------------ OneHotEncoder
def test_one_hot_encoder(tmp_path):
    train = Table.from_rows([(0.0,), (1.0,), (2.0,), (0.0,)], ["input"])
    pred = Table.from_rows([(0.0,), (1.0,), (2.0,)], ["input"])
    est = OneHotEncoder().set_input_cols("input").set_output_cols("output")
    assert est.get_drop_last() is True
    model = est.fit(train)
    p = str(tmp_path / "ohe")
    model.save(p)
    model = OneHotEncoderModel.load(p)
    out = model.transform(pred)[0].get_list("output")
    assert out == [Vectors.sparse(2, [0], [1.0]), Vectors.sparse(2, [1], [1.0]), Vectors.sparse(2, [], [])]
    assert model.get_model_data()[0].rows() == [(0, 2)]
    out2 = est.set_drop_last(False).fit(train).transform(pred)[0].get_list("output")
    assert out2 == [Vectors.sparse(3, [0], [1.0]), Vectors.sparse(3, [1], [1.0]), Vectors.sparse(3, [2], [1.0])]
    with pytest.raises(ValueError, match="indexed integer"):
        est.fit(Table.from_rows([(1.5,)], ["input"]))
    with pytest.raises(ValueError, match="Negative"):
        est.fit(Table.from_rows([(-1.0,)], ["input"]))
    with pytest.raises(ValueError):
        OneHotEncoder().set_input_cols("input").set_output_cols("output").set_handle_invalid("skip").fit(train)


def test_one_hot_encoder_model_data_bytes(tmp_path):
    model = OneHotEncoder().set_input_cols("a", "b").set_output_cols("x", "y").fit(
        Table.from_rows([(0, 3), (2, 1)], ["a", "b"]))
    p = str(tmp_path / "ohe2")
    model.save(p)
    import os
    raw = open(os.path.join(rw.data_path(p), "part-0-0"), "rb").read()
    assert raw == bytes([0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 1, 0, 0, 0, 3])


# ------------------------------------------------------------------ StringIndexer
SI_TRAIN = [("a", 1.0), ("b", 1.0), ("b", 2.0), ("c", 0.0), ("d", 2.0), ("a", 2.0), ("b", 2.0), ("b", -1.0),
            ("a", -1.0), ("c", -1.0)]
SI_PRED = [("a", 2.0), ("b", 1.0), ("e", 2.0)]


def _si(order, hi="keep"):
    return StringIndexer().set_input_cols("input_col1", "input_col2").set_output_cols("output_col1", "output_col2") \
        .set_string_order_type(order).set_handle_invalid(hi)


@pytest.mark.parametrize("order,expected", [
    ("alphabetAsc", [("a", 2.0, 0.0, 3.0), ("b", 1.0, 1.0, 2.0), ("e", 2.0, 4.0, 3.0)]),
    ("alphabetDesc", [("a", 2.0, 3.0, 0.0), ("b", 1.0, 2.0, 1.0), ("e", 2.0, 4.0, 0.0)]),
    ("frequencyAsc", [("a", 2.0, 2.0, 3.0), ("b", 1.0, 3.0, 1.0), ("e", 2.0, 4.0, 3.0)]),
    ("frequencyDesc", [("a", 2.0, 1.0, 0.0), ("b", 1.0, 0.0, 2.0), ("e", 2.0, 4.0, 0.0)]),
])
def test_string_indexer_orders(order, expected):
    train = Table.from_rows(SI_TRAIN, ["input_col1", "input_col2"])
    pred = Table.from_rows(SI_PRED, ["input_col1", "input_col2"])
    out = _si(order).fit(train).transform(pred)[0]
    assert out.column_names == ["input_col1", "input_col2", "output_col1", "output_col2"]
    got = [(r[0], float(r[1]), float(r[2]), float(r[3])) for r in out.rows()]
    assert got == expected


def test_string_indexer_arbitrary_skip_error_save(tmp_path):
    train = Table.from_rows(SI_TRAIN, ["input_col1", "input_col2"])
    pred = Table.from_rows(SI_PRED, ["input_col1", "input_col2"])
    est = StringIndexer().set_input_cols("input_col1", "input_col2").set_output_cols("o1", "o2")
    assert est.get_string_order_type() == "arbitrary" and est.get_handle_invalid() == "error"
    model = est.fit(train)
    arrays = model.get_model_data()[0].rows()[0][0]
    assert sorted(arrays[0]) == ["a", "b", "c", "d"] and sorted(arrays[1]) == ["-1.0", "0.0", "1.0", "2.0"]
    with pytest.raises(RuntimeError, match="unseen string: e"):
        model.transform(pred)
    skip = _si("alphabetAsc", "skip").fit(train).transform(pred)[0]
    assert [(r[0], float(r[2]), float(r[3])) for r in skip.rows()] == [("a", 0.0, 3.0), ("b", 1.0, 2.0)]
    m = _si("alphabetAsc").fit(train)
    assert m.get_model_data()[0].rows()[0][0] == [["a", "b", "c", "d"], ["-1.0", "0.0", "1.0", "2.0"]]
    p = str(tmp_path / "si")
    m.save(p)
    m2 = StringIndexerModel.load(p)
    assert m2.get_model_data()[0].rows()[0][0] == [["a", "b", "c", "d"], ["-1.0", "0.0", "1.0", "2.0"]]
    got = [(float(r[2]), float(r[3])) for r in m2.transform(pred)[0].rows()]
    assert got == [(0.0, 3.0), (1.0, 2.0), (4.0, 3.0)]


def test_index_to_string(tmp_path):
    md = StringIndexerModel.make_model_data_table([([["a", "b", "c", "d"], [-1.0, 0.0, 1.0, 2.0]],)])
    model = IndexToStringModel().set_input_cols("input_col1", "input_col2") \
        .set_output_cols("output_col1", "output_col2").set_model_data(md)
    pred = Table.from_rows([(0, 3), (1, 2)], ["input_col1", "input_col2"])
    out = model.transform(pred)[0]
    assert out.column_names == ["input_col1", "input_col2", "output_col1", "output_col2"]
    assert [(int(r[0]), int(r[1]), r[2], r[3]) for r in out.rows()] == [(0, 3, "a", "2.0"), (1, 2, "b", "1.0")]
    assert model.get_model_data()[0].rows()[0][0][1] == ["-1.0", "0.0", "1.0", "2.0"]
    p = str(tmp_path / "its")
    model.save(p)
    out2 = IndexToStringModel.load(p).transform(pred)[0]
    assert out2.get_list("output_col2") == ["2.0", "1.0"]
    with pytest.raises(RuntimeError, match="unseen index"):
        model.transform(Table.from_rows([(7, 0)], ["input_col1", "input_col2"]))


def test_java_number_strings():
    assert [java_number_to_string(v) for v in (1, 2.0, -1.0, 1e7, 1e-4, 0.5)] == \
        ["1", "2.0", "-1.0", "1.0E7", "1.0E-4", "0.5"]


# ------------------------------------------------------------------ VectorIndexer
VI_TRAIN = [(1, 1), (2, -1), (3, 1), (4, 0), (5, 0)]
VI_PRED = [(0, 2), (0, 0), (0, -1)]


def _vt(rows):
    return Table.from_rows([(Vectors.dense(*r),) for r in rows], ["input"])


def test_vector_indexer(tmp_path):
    vi = VectorIndexer()
    assert vi.get_max_categories() == 20
    model = vi.set_handle_invalid("keep").fit(_vt(VI_TRAIN))
    p = str(tmp_path / "vi")
    model.save(p)
    out = [arr(v).tolist() for v in VectorIndexerModel.load(p).transform(_vt(VI_PRED))[0].get_list("output")]
    assert sorted(out, key=lambda x: x[1]) == [[5, 0], [5, 1], [5, 3]]
    m3 = VectorIndexer().set_max_categories(3).fit(_vt(VI_TRAIN))
    assert m3.get_model_data()[0].rows()[0][0] == {1: {-1.0: 1, 0.0: 0, 1.0: 2}}
    with pytest.raises(RuntimeError, match="unseen double"):
        m3.transform(_vt(VI_PRED))
    skip = m3.set_handle_invalid("skip").transform(_vt(VI_PRED))[0]
    assert [arr(v).tolist() for v in skip.get_list("output")] == [[0, 0], [0, 1]]


def test_vector_indexer_sparse():
    t = Table.from_rows([(Vectors.sparse(3, [0], [5.0]),), (Vectors.sparse(3, [2], [-2.0]),)], ["input"])
    out = VectorIndexer().fit(t).transform(t)[0].get_list("output")
    # col0 {0->0, 5->1}; col1 {0->0}; col2 {0->0, -2->1} (0 is forced to index 0)
    assert [arr(v).tolist() for v in out] == [[1, 0, 0], [0, 0, 1]]


# ------------------------------------------------------------------ KBinsDiscretizer
KB_TRAIN = [(1, 10, 0), (1, 10, 0), (1, 10, 0), (4, 10, 0), (5, 10, 0), (6, 10, 0), (7, 10, 0), (10, 10, 0),
            (13, 10, 3)]
KB_PRED = [(-1, 0, 0), (1, 1, 1), (1.5, 1, 2), (5, 2, 3), (7.25, 3, 4), (13, 4, 5), (15, 4, 6)]


@pytest.mark.parametrize("strategy,expected", [
    ("uniform", [(0, 0, 0), (0, 0, 1), (0, 0, 2), (1, 0, 2), (1, 0, 2), (2, 0, 2), (2, 0, 2)]),
    ("quantile", [(0, 0, 0), (0, 0, 0), (0, 0, 0), (1, 0, 0), (2, 0, 0), (2, 0, 0), (2, 0, 0)]),
    ("kmeans", [(0, 0, 0), (0, 0, 1), (0, 0, 2), (1, 0, 2), (1, 0, 2), (2, 0, 2), (2, 0, 2)]),
])
def test_kbins(strategy, expected, tmp_path):
    kb = KBinsDiscretizer()
    assert (kb.get_num_bins(), kb.get_strategy(), kb.get_sub_samples()) == (5, "quantile", 200000)
    model = kb.set_num_bins(3).set_strategy(strategy).fit(_vt(KB_TRAIN))
    p = str(tmp_path / "kb")
    model.save(p)
    out = [tuple(arr(v).tolist()) for v in KBinsDiscretizerModel.load(p).transform(_vt(KB_PRED))[0].get_list("output")]
    assert sorted(out) == sorted(tuple(float(x) for x in e) for e in expected)


def test_kbins_model_data():
    model = KBinsDiscretizer().set_num_bins(3).set_strategy("uniform").fit(_vt(KB_TRAIN))
    edges = model.get_model_data()[0].rows()[0][0]
    np.testing.assert_allclose(edges[0], [1.0, 5.0, 9.0, 13.0])
    np.testing.assert_allclose(edges[1], [4.9e-324, 1.7976931348623157e308])
    np.testing.assert_allclose(edges[2], [0.0, 1.0, 2.0, 3.0])


# ------------------------------------------------------------------ Imputer
IM_ROWS = [(float("nan"), 9.0, 1), (1.0, 9.0, None), (1.5, 7.0, 1), (1.5, float("nan"), 2), (4.0, 5.0, 4),
           (None, 4.0, None)]
IM_EXPECTED = {
    "mean": [(2.0, 9.0, 1.0), (1.0, 9.0, 2.0), (1.5, 7.0, 1.0), (1.5, 6.8, 2.0), (4.0, 5.0, 4.0), (2.0, 4.0, 2.0)],
    "median": [(1.5, 9.0, 1.0), (1.0, 9.0, 1.0), (1.5, 7.0, 1.0), (1.5, 7.0, 2.0), (4.0, 5.0, 4.0), (1.5, 4.0, 1.0)],
    "most_frequent": [(1.5, 9.0, 1.0), (1.0, 9.0, 1.0), (1.5, 7.0, 1.0), (1.5, 9.0, 2.0), (4.0, 5.0, 4.0),
                      (1.5, 4.0, 1.0)],
}


@pytest.mark.parametrize("strategy", ["mean", "median", "most_frequent"])
def test_imputer(strategy, tmp_path):
    t = Table.from_rows(IM_ROWS, ["f1", "f2", "f3"])
    im = Imputer().set_input_cols("f1", "f2", "f3").set_output_cols("o1", "o2", "o3")
    assert math.isnan(im.get_missing_value())
    model = im.set_strategy(strategy).fit(t)
    p = str(tmp_path / "im")
    model.save(p)
    out = ImputerModel.load(p).transform(t)[0]
    assert out.column_names == ["f1", "f2", "f3", "o1", "o2", "o3"]
    got = [tuple(float(x) for x in r[3:]) for r in out.rows()]
    np.testing.assert_allclose(got, IM_EXPECTED[strategy], atol=1e-5)


def test_imputer_model_data_and_missing_value():
    t = Table.from_rows(IM_ROWS, ["f1", "f2", "f3"])
    model = Imputer().set_input_cols("f1", "f2", "f3").set_output_cols("o1", "o2", "o3").fit(t)
    (sur,), = model.get_model_data()[0].rows()
    assert abs(sur["f1"] - 2.0) < 1e-5 and abs(sur["f2"] - 6.8) < 1e-5 and abs(sur["f3"] - 2.0) < 1e-5
    t2 = Table.from_rows([(1.0,), (3.0,), (5.0,)], ["x"])
    m2 = Imputer().set_input_cols("x").set_output_cols("y").set_missing_value(1.0).fit(t2)
    assert m2.transform(t2)[0].get_list("y") == [4.0, 3.0, 5.0]


def _spmd_encoders(rank, world):
    train = Table.from_rows(SI_TRAIN, ["input_col1", "input_col2"]).partition(rank, world)
    si = _si("frequencyDesc").fit(train).get_model_data()[0].rows()[0][0]
    kb = KBinsDiscretizer().set_num_bins(3).set_strategy("uniform").fit(_vt(KB_TRAIN).partition(rank, world))
    im = Imputer().set_input_cols("f1", "f2", "f3").set_output_cols("o1", "o2", "o3").set_strategy("median") \
        .fit(Table.from_rows(IM_ROWS, ["f1", "f2", "f3"]).partition(rank, world))
    vi = VectorIndexer().set_max_categories(3).fit(_vt(VI_TRAIN).partition(rank, world))
    oh = OneHotEncoder().set_input_cols("input").set_output_cols("output").fit(
        Table.from_rows([(0.0,), (1.0,), (2.0,), (0.0,)], ["input"]).partition(rank, world))
    return (si, [list(e) for e in kb.get_model_data()[0].rows()[0][0]], im.get_model_data()[0].rows()[0][0],
            vi.get_model_data()[0].rows()[0][0], oh.get_model_data()[0].rows())


def test_encoders_distributed():
    for si, kb, im, vi, oh in run_spmd(_spmd_encoders, 2):
        assert [x for x in si[0] if x in ("a", "b")] == ["b", "a"] and si[1][0] in ("2.0", "-1.0")
        np.testing.assert_allclose(kb[0], [1.0, 5.0, 9.0, 13.0])
        assert im == {"f1": 1.5, "f2": 7.0, "f3": 1.0}
        assert vi == {1: {-1.0: 1, 0.0: 0, 1.0: 2}}
        assert oh == [(0, 2)]
