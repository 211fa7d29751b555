"""Native string tables (ops/csrc/host/strtab.cpp via utils/strtable.py) and the high-cardinality
string paths built on them: String.compareTo order, HashMap iteration order, hash-join lookup,
batched regex splitting — each against the per-string Python reference."""
import random
import re

import numpy as np
import torch

from flink_ml_amd import Table
from flink_ml_amd.models.feature.encoders import IndexToStringModel, StringIndexer
from flink_ml_amd.models.feature.text import batched_java_split, java_split
from flink_ml_amd.table import StringColumn
from flink_ml_amd.utils.java import java_hashmap_order, java_string_hash
from flink_ml_amd.utils.strtable import StrTable, hashmap_order_from_hashes

WORDS = ["b", "a", "ab", "", "zz", "a", "\U0001F600x", "é", "Ab", "a\u0000"]


def test_table_ops_match_python():
    t = StrTable.from_strings(WORDS)
    assert t.java_hashes().tolist() == [java_string_hash(w) for w in WORDS]
    assert [WORDS[i] for i in t.argsort()] == sorted(WORDS, key=lambda s: s.encode("utf-16-be"))
    assert [WORDS[i] for i in t.argsort(True)] == sorted(WORDS, key=lambda s: s.encode("utf-16-be"), reverse=True)
    assert t.first_of_equal().tolist() == [0, 1, 2, 3, 4, 1, 6, 7, 8, 9]
    q = StrTable.from_strings(["a", "nope", "\U0001F600x", ""])
    assert t.lookup(q).tolist() == [1, -1, 6, 3]
    sub = StrTable(t.units, t.offs).take(np.array([6, 7, 0, 3]))
    assert sub.strings() == ["\U0001F600x", "é", "b", ""]
    assert StrTable.concat([sub, t.take(np.array([2]))]).strings() == ["\U0001F600x", "é", "b", "", "ab"]
    h = t.hash64()
    assert h[1] == h[5] and len(set(h.tolist())) == 9


def test_hashmap_order_matches_reference_rule():
    rnd = random.Random(3)
    ws = ["%d" % rnd.randrange(10 ** 9) for _ in range(20000)]
    for n in (1, 12, 13, 300, 20000):
        order = hashmap_order_from_hashes(StrTable.from_strings(ws[:n]).java_hashes())
        assert [ws[i] for i in order] == java_hashmap_order(ws[:n])


def test_batched_regex_split_matches_java_split():
    rnd = random.Random(1)
    strs = ["".join(rnd.choice("ab1 1\tB") for _ in range(rnd.randrange(0, 9))) for _ in range(5000)]
    strs += ["", "1", "11", "1a", "a1", "A11B"]
    for p, low in (("1+", True), ("\\s+", False), ("1", True), ("[ab]", False)):
        ntok, tok = batched_java_split(strs, re.compile(p), low)
        offs = np.concatenate([[0], np.cumsum(ntok)])
        for i, s in enumerate(strs):
            assert list(tok[offs[i]:offs[i + 1]]) == java_split(p, s.lower() if low else s), (p, s)
    # patterns that are not safe across string boundaries fall back to the per-string path
    for p in ("^a", "(1)", "a*", "\\b1"):
        assert batched_java_split(strs, re.compile(p), False) is None


def test_string_indexer_high_cardinality_orders_and_index_to_string():
    rnd = random.Random(7)
    words = ["w%d" % rnd.randrange(30000) for _ in range(60000)]
    t = Table({"c": StringColumn.from_list(words)})
    counts = {}
    for w in words:
        counts[w] = counts.get(w, 0) + 1
    hm = java_hashmap_order(list(counts))
    refs = {"alphabetAsc": sorted(counts, key=lambda s: s.encode("utf-16-be")),
            "alphabetDesc": sorted(counts, key=lambda s: s.encode("utf-16-be"), reverse=True),
            "frequencyDesc": sorted(hm, key=lambda k: -counts[k]),
            "frequencyAsc": sorted(hm, key=lambda k: counts[k]), "arbitrary": hm}
    for order, ref in refs.items():
        m = StringIndexer().set_input_cols("c").set_output_cols("i").set_string_order_type(order).fit(t)
        arr = m.get_model_data()[0].rows()[0][0][0]
        assert arr == ref, order
        idx = m.transform(t)[0].column("i")
        pos = {w: i for i, w in enumerate(arr)}
        assert idx.tolist() == [float(pos[w]) for w in words]
        back = IndexToStringModel().set_input_cols("i").set_output_cols("s").set_model_data(
            m.get_model_data()[0]).transform(m.transform(t)[0])[0].column("s")
        assert isinstance(back, StringColumn) and back.to_list() == words
    # a later duplicate in a model array wins, like HashMap.put in array order
    md = StringIndexer().set_input_cols("c").set_output_cols("i").fit(t).get_model_data()[0]
    from flink_ml_amd.models.feature.encoders import StringIndexerModel

    dup = StringIndexerModel().set_input_cols("c").set_output_cols("i").set_model_data(
        StringIndexerModel.make_model_data_table([([["x", "y", "x"]],)]))
    out = dup.transform(Table({"c": StringColumn.from_list(["x", "y"])}))[0].column("i")
    assert out.tolist() == [2.0, 1.0]
    assert md is not None and torch.is_tensor(out)


def test_native_class_tokenizer_matches_java_split():
    """RegexTokenizer's native path for one-character patterns (optionally `X+`) equals
    String.split + minTokenLength on every string; other patterns are not taken."""
    from flink_ml_amd.models.feature.text import native_class_tokens, simple_class_pattern

    rnd = random.Random(3)
    strs = ["".join(rnd.choice("ab1 1\tB.,") for _ in range(rnd.randrange(0, 10))) for _ in range(3000)]
    strs += ["", "1", "11", "1a", "a1", "A11B", " x ", "  "]
    for p in ("1+", "1", "\\s+", "\\s", "[ab]+", "[^a-z]", ".", "\\.", "a|b"):
        table, plus = simple_class_pattern(p)
        for low in (True, False):
            for mn in (0, 1, 2):
                ntok, ids, vocab = native_class_tokens(strs, table, plus, low, mn)
                offs = np.concatenate([[0], np.cumsum(ntok)])
                for i, s in enumerate(strs):
                    ref = [x for x in java_split(p, s.lower() if low else s) if len(x) >= mn]
                    assert [vocab[j] for j in ids[offs[i]:offs[i + 1]]] == ref, (p, low, mn, s)
    for p in ("x*", "ab", "1{2}", "^a", "(1)+"):
        assert simple_class_pattern(p) is None
    assert native_class_tokens(["é1"], *simple_class_pattern("1"), True, 1) is None  # non-ASCII: Python path
