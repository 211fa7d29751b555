"""Stateless vector transformers against the reference's published expectations
(flink-ml-python/.../feature/tests/test_{binarizer,bucketizer,dct,elementwiseproduct,interaction,
normalizer,polynomialexpansion,vectorassembler,vectorslicer}.py and the Java tests)."""
import math

import numpy as np
import pytest
import torch

from flink_ml_amd import Table, Vectors
from flink_ml_amd.models import (DCT, Binarizer, Bucketizer, ElementwiseProduct, Interaction, Normalizer,
                                 PolynomialExpansion, VectorAssembler, VectorSlicer)


def arr(v):
    return np.asarray(v.to_array()) if hasattr(v, "to_array") else np.asarray(v)


def roundtrip(stage, tmp_path, name):
    p = str(tmp_path / name)
    stage.save(p)
    return type(stage).load(p)


def test_binarizer(tmp_path):
    t = Table.from_rows([
        (1, Vectors.dense(1, 2), Vectors.sparse(17, [0, 3, 9], [1.0, 2.0, 7.0])),
        (2, Vectors.dense(2, 1), Vectors.sparse(17, [0, 2, 14], [5.0, 4.0, 1.0])),
        (3, Vectors.dense(5, 18), Vectors.sparse(17, [0, 11, 12], [2.0, 4.0, 4.0]))], ["f0", "f1", "f2"])
    b = Binarizer().set_input_cols("f0", "f1", "f2").set_output_cols("of0", "of1", "of2").set_thresholds(1.0, 1.5, 2.5)
    assert b.get_input_cols() == ("f0", "f1", "f2") and b.get_thresholds() == (1.0, 1.5, 2.5)
    out = roundtrip(b, tmp_path, "bin").transform(t)[0]
    assert out.column_names == ["f0", "f1", "f2", "of0", "of1", "of2"]
    assert list(out.scalars("of0").tolist()) == [0.0, 1.0, 1.0]
    exp1 = [(0.0, 1.0), (1.0, 0.0), (1.0, 1.0)]
    exp2 = [Vectors.sparse(17, [9], [1.0]), Vectors.sparse(17, [0, 2], [1.0, 1.0]),
            Vectors.sparse(17, [11, 12], [1.0, 1.0])]
    for i, (v1, v2) in enumerate(zip(out.get_list("of1"), out.get_list("of2"))):
        np.testing.assert_allclose(arr(v1), exp1[i])
        assert v2.size() == 17
        np.testing.assert_allclose(arr(v2), arr(exp2[i]))


BUCKET_SPLITS = ((-0.5, 0.0, 0.5), (-1.0, 0.0, 2.0), (float("-inf"), 10.0, float("inf")))


def _bucket_table():
    return Table.from_rows([(1, -0.5, 0.0, 1.0), (2, float("-inf"), 1.0, float("inf")),
                            (3, float("nan"), -0.5, -0.5)], ["id", "f1", "f2", "f3"])


@pytest.mark.parametrize("mode,expected", [("keep", [(1, 0, 1, 0), (2, 2, 1, 1), (3, 2, 0, 0)]),
                                           ("skip", [(1, 0, 1, 0)])])
def test_bucketizer(mode, expected, tmp_path):
    b = Bucketizer().set_input_cols("f1", "f2", "f3").set_output_cols("o1", "o2", "o3")
    assert b.get_handle_invalid() == "error"
    b.set_handle_invalid(mode).set_splits_array(BUCKET_SPLITS)
    assert b.get_splits_array() == BUCKET_SPLITS
    out = roundtrip(b, tmp_path, "bk").transform(_bucket_table())[0]
    assert out.column_names == ["id", "f1", "f2", "f3", "o1", "o2", "o3"]
    got = [(int(r[0]), int(r[4]), int(r[5]), int(r[6])) for r in out.rows()]
    assert got == expected


def test_bucketizer_error():
    b = Bucketizer().set_input_cols("f1", "f2", "f3").set_output_cols("o1", "o2", "o3") \
        .set_splits_array(BUCKET_SPLITS)
    with pytest.raises(RuntimeError, match="invalid"):
        b.transform(_bucket_table())


def _tol(fp64_tol: float) -> float:
    """The fp64 tolerance on the host path; on a GPU host the stages compute in the fp32 policy."""
    from flink_ml_amd import config

    return fp64_tol if config.compute_dtype() == torch.float64 else max(fp64_tol, 1e-6)


def test_dct(tmp_path):
    t = Table.from_rows([(Vectors.dense(1.0, 1.0, 1.0, 1.0),), (Vectors.dense(1.0, 0.0, -1.0, 0.0),)], ["input"])
    d = DCT()
    assert d.get_inverse() is False
    out = roundtrip(d, tmp_path, "dct").transform(t)[0]
    assert out.column_names == ["input", "output"]
    res = [arr(v) for v in out.get_list("output")]
    np.testing.assert_allclose(res[0], [2.0, 0.0, 0.0, 0.0], atol=1e-3)
    np.testing.assert_allclose(res[1], [0.0, 0.924, 1.0, -0.383], atol=1e-3)
    inv = DCT().set_inverse(True).set_input_col("output").set_output_col("back").transform(out)[0]
    for a, b in zip(inv.get_list("back"), inv.get_list("input")):
        np.testing.assert_allclose(arr(a), arr(b), atol=_tol(1e-12))


def test_elementwise_product(tmp_path):
    t = Table.from_rows([(0, Vectors.dense(2.1, 3.1)), (1, Vectors.dense(1.1, 3.3)),
                         (2, Vectors.sparse(2, [1], [2.0]))], ["id", "vec"])
    e = ElementwiseProduct().set_input_col("vec").set_output_col("output_vec").set_scaling_vec(Vectors.dense(1.1, 1.1))
    assert e.get_scaling_vec() == Vectors.dense(1.1, 1.1)
    out = roundtrip(e, tmp_path, "ep").transform(t)[0]
    got = out.get_list("output_vec")
    np.testing.assert_allclose(arr(got[0]), [2.31, 3.41], atol=1e-7)
    np.testing.assert_allclose(arr(got[1]), [1.21, 3.63], atol=1e-7)
    np.testing.assert_allclose(arr(got[2]), [0.0, 2.2], atol=1e-7)


def test_interaction(tmp_path):
    t = Table.from_rows([(1, Vectors.dense(1, 2), Vectors.dense(3, 4)), (2, Vectors.dense(2, 8), Vectors.dense(3, 4))],
                        ["f0", "f1", "f2"])
    it = Interaction().set_input_cols("f0", "f1", "f2").set_output_col("interaction_vec")
    out = roundtrip(it, tmp_path, "ia").transform(t)[0]
    got = out.get_list("interaction_vec")
    np.testing.assert_allclose(arr(got[0]), [3.0, 4.0, 6.0, 8.0], atol=1e-5)
    np.testing.assert_allclose(arr(got[1]), [12.0, 16.0, 48.0, 64.0], atol=1e-5)


def test_normalizer(tmp_path):
    t = Table.from_rows([(Vectors.dense(2.1, 3.1, 2.3, 3.4, 5.3, 5.1),), (Vectors.dense(2.3, 4.1, 1.3, 2.4, 5.1, 4.1),)],
                        ["intput_vec"])
    n = Normalizer()
    assert n.get_p() == 2.0
    n.set_input_col("intput_vec").set_output_col("output_vec").set_p(1.5)
    assert isinstance(n.get_p(), float)
    out = roundtrip(n, tmp_path, "nm").transform(t)[0]
    exp = [[0.17386300895299714, 0.25665491797823387, 0.19042139075804446, 0.28149249068580484, 0.43879711783375464,
            0.42223873602870726],
           [0.20785190042726007, 0.3705186051094636, 0.11748150893714701, 0.2168889395762714, 0.4608889965995767,
            0.3705186051094636]]
    for v, e in zip(out.get_list("output_vec"), exp):
        np.testing.assert_allclose(arr(v), e, rtol=_tol(1e-12))


def test_normalizer_sparse_and_inf():
    t = Table.from_rows([(Vectors.sparse(5, [1, 4], [3.0, -4.0]),)], ["input"])
    out = Normalizer().set_p(float("inf")).transform(t)[0].get_list("output")[0]
    assert out.size() == 5 and list(out.indices) == [1, 4]
    np.testing.assert_allclose(out.values, [0.75, -1.0])


def test_polynomial_expansion(tmp_path):
    t = Table.from_rows([(Vectors.dense(1.0, 2.0),), (Vectors.dense(2.0, 3.0),)], ["intput_vec"])
    pe = PolynomialExpansion()
    assert pe.get_degree() == 2
    pe.set_input_col("intput_vec").set_output_col("output_vec")
    out = roundtrip(pe, tmp_path, "pe").transform(t)[0]
    got = [arr(v).tolist() for v in out.get_list("output_vec")]
    assert got == [[1.0, 1.0, 2.0, 2.0, 4.0], [2.0, 4.0, 3.0, 6.0, 9.0]]
    # degree 3 on 3 features has C(3+3,3)-1 = 19 terms
    t3 = Table.from_rows([(Vectors.dense(2.0, 3.0, 5.0),)], ["input"])
    v3 = arr(PolynomialExpansion().set_degree(3).transform(t3)[0].get_list("output")[0])
    assert len(v3) == 19 and sorted(v3.tolist()) == sorted(
        [2 ** a * 3 ** b * 5 ** c for a in range(4) for b in range(4) for c in range(4) if 0 < a + b + c <= 3])


def test_vector_assembler(tmp_path):
    t = Table.from_rows([(0, Vectors.dense(2.1, 3.1), 1.0, Vectors.sparse(5, [3], [1.0])),
                         (1, Vectors.dense(2.1, 3.1), 1.0, Vectors.sparse(5, [1, 2, 3, 4], [1.0, 2.0, 3.0, 4.0]))],
                        ["id", "vec", "num", "sparse_vec"])
    va = VectorAssembler().set_input_cols("vec", "num", "sparse_vec").set_output_col("assembled_vec") \
        .set_input_sizes(2, 1, 5).set_handle_invalid("keep")
    assert va.get_input_sizes() == (2, 1, 5)
    out = roundtrip(va, tmp_path, "va").transform(t)[0]
    got = out.get_list("assembled_vec")
    assert got[0] == Vectors.sparse(8, [0, 1, 2, 6], [2.1, 3.1, 1.0, 1.0])
    assert got[1] == Vectors.dense(2.1, 3.1, 1.0, 0.0, 1.0, 2.0, 3.0, 4.0)


def test_vector_assembler_invalid_size():
    t = Table.from_rows([(Vectors.dense(2.1, 3.1), 1.0)], ["vec", "num"])
    va = VectorAssembler().set_input_cols("vec", "num").set_output_col("o").set_input_sizes(3, 1)
    with pytest.raises(Exception):
        va.transform(t)
    out = va.set_handle_invalid("skip").transform(t)[0]
    assert out.num_rows == 0


def test_vector_slicer(tmp_path):
    t = Table.from_rows([(1, Vectors.dense(2.1, 3.1, 1.2, 2.1)), (2, Vectors.dense(2.3, 2.1, 1.3, 1.2))], ["id", "vec"])
    vs = VectorSlicer().set_input_col("vec").set_output_col("slice_vec").set_indices(0, 1, 2)
    assert vs.get_indices() == (0, 1, 2)
    out = roundtrip(vs, tmp_path, "vs").transform(t)[0]
    got = out.get_list("slice_vec")
    assert got[0] == Vectors.dense(2.1, 3.1, 1.2) and got[1] == Vectors.dense(2.3, 2.1, 1.3)
    with pytest.raises(ValueError):
        VectorSlicer().set_indices(1, 1)
