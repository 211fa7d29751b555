"""Dictionary-encoded string-array columns (``StringArrayColumn``): the device fast paths of the
string-array stages must give exactly what the per-row host path gives on the same rows as plain
lists (StopWordsRemover.java, HashingTF.java, CountVectorizer(Model).java semantics)."""
import numpy as np
import pytest
import torch

from flink_ml_amd import Table
from flink_ml_amd.lib.feature.countvectorizer import CountVectorizer
from flink_ml_amd.lib.feature.hashingtf import HashingTF
from flink_ml_amd.lib.feature.stopwordsremover import StopWordsRemover
from flink_ml_amd.table import StringArrayColumn

ROWS = [["The", "a", "quick", "fox"], [], ["fox", "fox", "The", "zebra", "a"], ["b", "quick"],
        ["a", "a", "a"], ["x", "y", "b", "fox", "quick", "quick"]]


def _both():
    return Table({"input": [list(r) for r in ROWS]}), Table({"input": StringArrayColumn.from_lists(ROWS)})


def _dense(col, n):
    return [v.to_array().tolist() for v in Table({"c": col}, num_rows=n).get_list("c")]


def test_column_behaves_like_list_of_lists():
    c = StringArrayColumn.from_lists(ROWS)
    assert len(c) == len(ROWS)
    assert c.to_lists() == ROWS
    assert c[2] == ROWS[2] and c[-1] == ROWS[-1]
    assert c[1:4].to_lists() == ROWS[1:4]
    t = Table({"input": c, "id": torch.arange(len(ROWS))})
    assert t.slice(2, 5).get_list("input") == ROWS[2:5]
    assert t.take(torch.tensor([5, 0])).get_list("input") == [ROWS[5], ROWS[0]]
    assert Table.concat([t.slice(0, 2), t.slice(2, 6)]).get_list("input") == ROWS
    dense = StringArrayColumn.from_dense_codes(torch.tensor([[0, 1], [1, 1]]), ["u", "v"])
    assert dense.to_lists() == [["u", "v"], ["v", "v"]]


def test_stopwords_remover_matches_host_path():
    tl, tc = _both()
    for cs in (False, True):
        st = StopWordsRemover().set_input_cols("input").set_output_cols("output").set_case_sensitive(cs)
        assert st.transform(tc)[0].get_list("output") == st.transform(tl)[0].get_list("output")
    # a slice (offsets not starting at 0) goes through the same path
    st = StopWordsRemover().set_input_cols("input").set_output_cols("output")
    assert st.transform(tc.slice(2, 6))[0].get_list("output") == st.transform(tl.slice(2, 6))[0].get_list("output")


def test_hashingtf_matches_host_path():
    tl, tc = _both()
    for binary in (False, True):
        h = HashingTF().set_num_features(64).set_binary(binary)
        a = h.transform(tl)[0].get_list("output")
        b = h.transform(tc)[0].get_list("output")
        assert [(v.indices.tolist(), v.values.tolist()) for v in a] == [(v.indices.tolist(), v.values.tolist()) for v in b]


def test_countvectorizer_fit_and_transform_match_host_path():
    tl, tc = _both()
    for min_tf, binary in ((1.0, False), (2.0, False), (0.3, True)):
        cv = CountVectorizer().set_min_tf(min_tf).set_binary(binary)
        ml, mc = cv.fit(tl), cv.fit(tc)
        vl = ml.get_model_data()[0].get_list("vocabulary")
        assert vl == mc.get_model_data()[0].get_list("vocabulary")
        a = ml.transform(tl)[0].get_list("output")
        b = mc.transform(tc)[0].get_list("output")
        assert [(v.size(), v.indices.tolist(), v.values.tolist()) for v in a] == \
               [(v.size(), v.indices.tolist(), v.values.tolist()) for v in b]


def test_generator_emits_dictionary_encoded_arrays():
    from flink_ml_amd.bench.generators import RandomStringArrayGenerator

    g = RandomStringArrayGenerator().set_col_names([["input"]]).set_num_values(50).set_array_size(7) \
        .set_num_distinct_values(10).set_seed(2)
    t = g.get_data()[0]
    col = t.column("input")
    assert isinstance(col, StringArrayColumn)
    rows = t.get_list("input")
    assert len(rows) == 50 and all(len(r) == 7 for r in rows)
    assert set(np.concatenate(rows)) <= {str(i) for i in range(10)}


def test_ngram_matches_host_path():
    from flink_ml_amd.lib.feature.ngram import NGram

    tl, tc = _both()
    for n in (1, 2, 3, 5):
        ng = NGram().set_n(n)
        got = ng.transform(tc)[0]
        assert isinstance(got.column("output"), StringArrayColumn)
        assert got.get_list("output") == ng.transform(tl)[0].get_list("output")
    ng = NGram().set_n(2)
    assert ng.transform(tc.slice(1, 5))[0].get_list("output") == ng.transform(tl.slice(1, 5))[0].get_list("output")


STRS = ["Hello World", "a  b\tc", "", "Hello World", "UPPER case  Words", "x"]


def test_string_column_behaves_like_list():
    from flink_ml_amd.table import StringColumn

    c = StringColumn.from_list(STRS)
    assert c.to_list() == STRS and list(c) == STRS and c[4] == STRS[4]
    t = Table({"s": c, "id": torch.arange(len(STRS))})
    assert t.slice(1, 4).get_list("s") == STRS[1:4]
    assert t.take(torch.tensor([5, 0, 3])).get_list("s") == [STRS[5], STRS[0], STRS[3]]
    assert t.filter(torch.tensor([True, False, True, False, False, True])).get_list("s") == [STRS[0], STRS[2], STRS[5]]


def test_tokenizers_match_host_path():
    from flink_ml_amd.lib.feature.regextokenizer import RegexTokenizer
    from flink_ml_amd.lib.feature.tokenizer import Tokenizer
    from flink_ml_amd.table import StringColumn

    tl, tc = Table({"input": list(STRS)}), Table({"input": StringColumn.from_list(STRS)})
    stages = [Tokenizer(), RegexTokenizer(), RegexTokenizer().set_gaps(False).set_pattern("\\w+").set_min_token_length(2),
              RegexTokenizer().set_to_lowercase(False)]
    for st in stages:
        got = st.transform(tc)[0]
        assert isinstance(got.column("output"), StringArrayColumn)
        assert got.get_list("output") == st.transform(tl)[0].get_list("output")


def test_stringindexer_matches_host_path():
    from flink_ml_amd.lib.feature.stringindexer import StringIndexer
    from flink_ml_amd.table import StringColumn

    vals = ["b", "a", "c", "a", "b", "a", "d"]
    tl = Table({"f": list(vals)})
    tc = Table({"f": StringColumn.from_list(vals)})
    for order in ("arbitrary", "frequencyDesc", "frequencyAsc", "alphabetDesc", "alphabetAsc"):
        si = StringIndexer().set_input_cols("f").set_output_cols("o").set_string_order_type(order)
        ml, mc = si.fit(tl), si.fit(tc)
        assert ml.get_model_data()[0].get_list("stringArrays") == mc.get_model_data()[0].get_list("stringArrays")
        assert ml.transform(tl)[0].get_list("o") == mc.transform(tc)[0].get_list("o")
    test = Table({"f": StringColumn.from_list(["a", "zz", "b"])})
    m = StringIndexer().set_input_cols("f").set_output_cols("o").set_handle_invalid("keep").fit(tc)
    ref = m.transform(Table({"f": ["a", "zz", "b"]}))[0].get_list("o")
    assert m.transform(test)[0].get_list("o") == ref
    m.set_handle_invalid("skip")
    assert m.transform(test)[0].num_rows == 2


@pytest.mark.gpu
def test_string_stages_run_on_device():
    """The same equivalences with the codes in HBM (the device gathers/scans/sorts are what run)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from flink_ml_amd import config

    assert config.compute_device().type == "cuda"
    test_stopwords_remover_matches_host_path()
    test_hashingtf_matches_host_path()
    test_countvectorizer_fit_and_transform_match_host_path()
    test_ngram_matches_host_path()
    test_tokenizers_match_host_path()
    test_stringindexer_matches_host_path()
    _, tc = _both()
    out = StopWordsRemover().set_input_cols("input").set_output_cols("output").transform(tc)[0].column("output")
    assert out.codes.device.type == "cuda"


def test_string_array_slice_of_slice_and_indexing():
    """slicing a sliced StringArrayColumn and indexing rows of a slice read the right codes."""
    from flink_ml_amd.table import StringArrayColumn

    rows = [["a", "b"], [], ["c"], ["d", "e", "f"], ["g"], ["h", "i"], []]
    col = StringArrayColumn.from_lists(rows)
    s1 = col[2:7]
    assert s1.to_lists() == rows[2:7]
    s2 = s1[1:4]
    assert s2.to_lists() == rows[3:6]
    assert [s2[i] for i in range(len(s2))] == rows[3:6]
    assert s1[3] == rows[5] and s1[-1] == rows[6]
    assert s2[1:2].to_lists() == [rows[4]]
