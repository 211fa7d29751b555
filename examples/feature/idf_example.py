"""Fits inverse document frequencies and rescales term-frequency vectors.

Run: python examples/feature/idf_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import IDF  # noqa: E402
data = Table.from_rows([(Vectors.dense(0, 1, 0, 2),), (Vectors.dense(0, 1, 2, 3),), (Vectors.dense(0, 1, 0, 0),)],
                       ["input"])
model = IDF().set_min_doc_freq(2).fit(data)
out = model.transform(data)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
