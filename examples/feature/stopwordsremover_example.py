"""Removes stop words from token sequences.

Run: python examples/feature/stopwordsremover_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import StopWordsRemover  # noqa: E402
data = Table.from_rows([(["test", "test"], ["test", "test"]), (["a", "b", "c", "d"], ["a", "b"]),
                        (["a", "the", "an"], ["a", "the", "test"]), (["A", "The", "AN"], ["A", "The", "TEST"]),
                        ([None, "a", "b"], [None, "a", "b"])], ["input", "input2"])
stage = StopWordsRemover().set_input_cols("input", "input2").set_output_cols("output", "output2")
out = stage.transform(data)[0]
for row in out.select("input", "input2", "output", "output2").rows():
    print("Input Values: %s \tOutput Values: %s" % (list(row[:2]), list(row[2:])))
