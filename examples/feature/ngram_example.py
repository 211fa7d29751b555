"""Turns token sequences into sequences of n-grams.

Run: python examples/feature/ngram_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import NGram  # noqa: E402
data = Table.from_rows([([],), (["a", "b", "c"],), (["a", "b", "c", "d"],)], ["input"])
out = NGram().set_n(2).set_input_col("input").set_output_col("output").transform(data)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
