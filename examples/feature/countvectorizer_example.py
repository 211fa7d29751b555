"""Builds a vocabulary from documents and turns them into term-count vectors.

Run: python examples/feature/countvectorizer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import CountVectorizer  # noqa: E402
data = Table.from_rows([(["a", "c", "b", "c"],), (["c", "d", "e"],), (["a", "b", "c"],), (["e", "f"],),
                        (["a", "c", "a"],)], ["input"])
model = CountVectorizer().fit(data)
out = model.transform(data)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
