"""Binarizes numeric and vector columns with per-column thresholds.

Run: python examples/feature/binarizer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import Binarizer  # noqa: E402
data = Table.from_rows([(1, Vectors.dense(3, 4)), (2, Vectors.dense(6, 2))], ["f0", "f1"])
stage = Binarizer().set_input_cols("f0", "f1").set_output_cols("of0", "of1").set_thresholds(1.5, 3.5)
out = stage.transform(data)[0]
for f0, f1, o0, o1 in out.select("f0", "f1", "of0", "of1").rows():
    print("Input Values: %s \tOutput Values: %s" % ([f0, f1], [o0, o1]))
