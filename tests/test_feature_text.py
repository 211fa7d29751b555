"""Text / hashing stages against the reference's expectations
(flink-ml-python/.../feature/tests/test_{tokenizer,regextokenizer,ngram,stopwordsremover,hashingtf,
feature_hasher,countvectorizer,idf}.py and LIBT/feature/CountVectorizerTest.java, IDFTest.java)."""
import numpy as np
import pytest

from flink_ml_amd import Table, Vectors
from flink_ml_amd.models import (IDF, CountVectorizer, CountVectorizerModel, FeatureHasher, HashingTF, IDFModel, NGram,
                                 RegexTokenizer, StopWordsRemover, Tokenizer)
from flink_ml_amd.ops import hashing
from tests.spmd import run_spmd


def roundtrip(stage, tmp_path, name):
    p = str(tmp_path / name)
    stage.save(p)
    return type(stage).load(p)


def test_tokenizers(tmp_path):
    t = Table.from_rows([("Test for tokenization.",), ("Te,st. punct",)], ["input"])
    exp = [["test", "for", "tokenization."], ["te,st.", "punct"]]
    assert roundtrip(Tokenizer(), tmp_path, "tok").transform(t)[0].get_list("output") == exp
    rt = RegexTokenizer()
    assert rt.get_min_token_length() == 1 and rt.get_gaps() is True and rt.get_to_lowercase() is True
    assert roundtrip(rt, tmp_path, "rt").transform(t)[0].get_list("output") == exp
    words = RegexTokenizer().set_gaps(False).set_pattern("\\w+").set_min_token_length(3).set_to_lowercase(False)
    assert words.transform(t)[0].get_list("output") == [["Test", "for", "tokenization"], ["punct"]]


def test_ngram(tmp_path):
    t = Table.from_rows([([],), (["a", "b", "c"],), (["a", "b", "c", "d"],)], ["input"])
    ng = NGram()
    assert ng.get_n() == 2
    out = roundtrip(ng, tmp_path, "ng").transform(t)[0].get_list("output")
    assert out == [[], ["a b", "b c"], ["a b", "b c", "c d"]]
    assert NGram().set_n(5).transform(t)[0].get_list("output") == [[], [], []]


def test_stop_words_remover(tmp_path):
    rows = [(["test", "test"], ["test", "test"]), (["a", "b", "c", "d"], ["b", "c", "d"]), (["a", "the", "an"], []),
            (["A", "The", "AN"], []), ([None], [None]), ([], [])]
    t = Table.from_rows(rows, ["raw", "expected"])
    r = StopWordsRemover()
    assert {"i", "would"} <= set(r.get_stop_words())
    assert r.get_locale() == StopWordsRemover.get_default_or_us() and r.get_case_sensitive() is False
    r.set_input_cols("raw").set_output_cols("filtered")
    out = roundtrip(r, tmp_path, "sw").transform(t)[0]
    assert out.column_names == ["raw", "expected", "filtered"]
    assert out.get_list("filtered") == out.get_list("expected")
    assert "en_US" in StopWordsRemover.get_available_locales()
    for lang in StopWordsRemover.SUPPORTED_LANGUAGES:
        assert len(StopWordsRemover.load_default_stop_words(lang)) > 0
    tr = StopWordsRemover.load_default_stop_words("turkish")
    assert {"acaba", "yani"} <= set(tr)
    with pytest.raises(ValueError):
        StopWordsRemover().set_locale("xx_YY")
    cs = StopWordsRemover().set_input_cols("raw").set_output_cols("f").set_case_sensitive(True).transform(t)[0]
    assert cs.get_list("f")[3] == ["A", "The", "AN"]


def test_hashing_tf(tmp_path):
    t = Table.from_rows([(["HashingTFTest", "Hashing", "Term", "Frequency", "Test"],),
                         (["HashingTFTest", "Hashing", "Hashing", "Test", "Test"],)], ["input"])
    h = HashingTF()
    assert h.get_binary() is False and h.get_num_features() == 262144
    out = roundtrip(h, tmp_path, "htf").transform(t)[0].get_list("output")
    assert out[0] == Vectors.sparse(262144, [67564, 89917, 113827, 131486, 228971], [1.0] * 5)
    assert out[1] == Vectors.sparse(262144, [67564, 131486, 228971], [1.0, 2.0, 2.0])
    ob = HashingTF().set_binary(True).transform(t)[0].get_list("output")
    assert ob[1] == Vectors.sparse(262144, [67564, 131486, 228971], [1.0, 1.0, 1.0])


def test_murmur3_matches_guava():
    # Guava Hashing.murmur3_32(0).hashUnencodedChars / hashInt reference values
    assert hashing.hash_strings(["HashingTFTest"]).shape == (1,)
    assert int(hashing.hash_ints([0])[0]) == 593689054
    assert int(hashing.hash_ints([1])[0]) == -68075478


def test_feature_hasher(tmp_path):
    t = Table.from_rows([(0, "a", 1.0, True), (1, "c", 1.0, False)], ["id", "f0", "f1", "f2"])
    fh = FeatureHasher()
    assert fh.get_num_features() == 262144
    fh.set_input_cols("f0", "f1", "f2").set_categorical_cols("f0", "f2").set_output_col("vec").set_num_features(1000)
    assert fh.get_categorical_cols() == ("f0", "f2")
    out = roundtrip(fh, tmp_path, "fh").transform(t)[0].get_list("vec")
    assert out[0] == Vectors.sparse(1000, [607, 635, 913], [1.0, 1.0, 1.0])
    assert out[1] == Vectors.sparse(1000, [242, 869, 913], [1.0, 1.0, 1.0])


CV_ROWS = [(1, ["a", "c", "b", "c"]), (2, ["c", "d", "e"]), (3, ["a", "b", "c"]), (4, ["e", "f"]), (5, ["a", "c", "a"])]


def _cv_table():
    return Table.from_rows(CV_ROWS, ["id", "input"])


def test_count_vectorizer_default(tmp_path):
    cv = CountVectorizer()
    assert cv.get_min_df() == 1.0 and cv.get_max_df() == float(2 ** 63 - 1) and cv.get_min_tf() == 1.0
    assert cv.get_vocabulary_size() == 1 << 18 and cv.get_binary() is False
    model = roundtrip(cv, tmp_path, "cv").fit(_cv_table())
    assert model.get_model_data()[0].column_names == ["vocabulary"]
    assert list(model.get_model_data()[0].rows()[0][0]) == ["c", "a", "b", "e", "d", "f"]
    out = roundtrip(model, tmp_path, "cvm").transform(_cv_table())[0]
    assert out.column_names == ["id", "input", "output"]
    assert out.get_list("output") == [
        Vectors.sparse(6, [0, 1, 2], [2.0, 1.0, 1.0]), Vectors.sparse(6, [0, 3, 4], [1.0, 1.0, 1.0]),
        Vectors.sparse(6, [0, 1, 2], [1.0, 1.0, 1.0]), Vectors.sparse(6, [3, 5], [1.0, 1.0]),
        Vectors.sparse(6, [0, 1], [1.0, 2.0])]
    m2 = CountVectorizerModel().set_model_data(*model.get_model_data())
    assert m2.transform(_cv_table())[0].get_list("output") == out.get_list("output")


@pytest.mark.parametrize("setup,expected", [
    (lambda c: c.set_min_df(2.0).set_max_df(4.0),
     [(4, [0, 1, 2], [2, 1, 1]), (4, [0, 3], [1, 1]), (4, [0, 1, 2], [1, 1, 1]), (4, [3], [1]), (4, [0, 1], [1, 2])]),
    (lambda c: c.set_min_df(0.4).set_max_df(0.8),
     [(4, [0, 1, 2], [2, 1, 1]), (4, [0, 3], [1, 1]), (4, [0, 1, 2], [1, 1, 1]), (4, [3], [1]), (4, [0, 1], [1, 2])]),
    (lambda c: c.set_min_tf(0.5),
     [(6, [0], [2]), (6, [], []), (6, [], []), (6, [3, 5], [1, 1]), (6, [1], [2])]),
    (lambda c: c.set_binary(True),
     [(6, [0, 1, 2], [1, 1, 1]), (6, [0, 3, 4], [1, 1, 1]), (6, [0, 1, 2], [1, 1, 1]), (6, [3, 5], [1, 1]),
      (6, [0, 1], [1, 1])]),
    (lambda c: c.set_vocabulary_size(2),
     [(2, [0, 1], [2, 1]), (2, [0], [1]), (2, [0, 1], [1, 1]), (2, [], []), (2, [0, 1], [1, 2])]),
])
def test_count_vectorizer_variants(setup, expected):
    model = setup(CountVectorizer()).fit(_cv_table())
    out = model.transform(_cv_table())[0].get_list("output")
    assert out == [Vectors.sparse(n, i, [float(x) for x in v]) for n, i, v in expected]


@pytest.mark.parametrize("mx,mn", [(0.1, 0.2), (1.0, 2.0), (1.0, 0.9), (0.1, 10.0)])
def test_count_vectorizer_invalid_df(mx, mn):
    with pytest.raises(Exception, match="maxDF must be >= minDF."):
        CountVectorizer().set_max_df(mx).set_min_df(mn).fit(_cv_table()).transform(_cv_table())


IDF_ROWS = [(Vectors.dense(0, 1, 0, 2),), (Vectors.dense(0, 1, 2, 3),), (Vectors.dense(0, 1, 0, 0),)]


def test_idf(tmp_path):
    t = Table.from_rows(IDF_ROWS, ["input"])
    idf = IDF()
    assert idf.get_min_doc_freq() == 0
    model = roundtrip(idf, tmp_path, "idf").fit(t)
    out = [v.to_array() for v in roundtrip(model, tmp_path, "idfm").transform(t)[0].get_list("output")]
    exp = [[0.0, 0.0, 0.0, 0.5753641], [0.0, 0.0, 1.3862943, 0.8630462], [0.0, 0.0, 0.0, 0.0]]
    np.testing.assert_allclose(out, exp, atol=1e-7)
    md = model.get_model_data()[0]
    assert md.column_names == ["idf", "docFreq", "numDocs"]
    (_, df, nd), = md.rows()
    assert nd == 3 and list(df) == [0, 3, 1, 2]
    out2 = [v.to_array() for v in IDF().set_min_doc_freq(2).fit(t).transform(t)[0].get_list("output")]
    np.testing.assert_allclose(out2, [[0, 0, 0, 0.5753641], [0, 0, 0, 0.8630462], [0, 0, 0, 0]], atol=1e-7)
    sp = Table.from_rows([(Vectors.sparse(4, [1, 3], [1.0, 2.0]),)], ["input"])
    outs = IDFModel().set_model_data(md).transform(sp)[0].get_list("output")[0]
    np.testing.assert_allclose(outs.to_array(), [0, 0, 0, 0.5753641], atol=1e-7)


def _spmd_text(rank, world):
    cv = CountVectorizer().fit(_cv_table().partition(rank, world))
    idf = IDF().fit(Table.from_rows(IDF_ROWS, ["input"]).partition(rank, world))
    (_, df, nd), = idf.get_model_data()[0].rows()
    return list(cv.get_model_data()[0].rows()[0][0]), list(df), nd


def test_text_distributed():
    for vocab, df, nd in run_spmd(_spmd_text, 2):
        assert vocab == ["c", "a", "b", "e", "d", "f"]
        assert df == [0, 3, 1, 2] and nd == 3


def test_count_vectorizer_document_frequency_paths_agree(monkeypatch):
    """The three document-frequency paths (presence bitmap, per-document segmented sort, global
    unique of (doc, term) keys) give the same vocabulary (ordered by document frequency)."""
    import random

    from flink_ml_amd.models.feature import text as tx
    from flink_ml_amd.models.feature.text import CountVectorizer
    from flink_ml_amd.table import StringArrayColumn

    rnd = random.Random(4)
    docs = [["t%d" % rnd.randrange(300) for _ in range(12)] for _ in range(400)]
    t = Table({"input": StringArrayColumn.from_lists(docs)})
    out = []
    for bitmap_max, seg in ((1 << 32, True), (0, True), (0, False)):
        monkeypatch.setattr(tx, "DF_BITMAP_MAX", bitmap_max)
        monkeypatch.setattr(tx, "DF_SEGMENTED_SORT", seg)
        m = CountVectorizer().set_min_df(3.0).set_max_df(200.0).fit(t)
        out.append(m.get_model_data()[0].rows()[0][0])
    assert out[0] == out[1] == out[2] and len(out[0]) > 100
