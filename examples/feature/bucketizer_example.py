"""Maps continuous columns to bucket indices given split points.

Run: python examples/feature/bucketizer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import Bucketizer  # noqa: E402
data = Table.from_rows([(-0.5, 0.0, 1.0, 0.0)], ["f1", "f2", "f3", "f4"])
splits = [[-0.5, 0.0, 0.5], [-1.0, 0.0, 2.0], [float("-inf"), 10.0, float("inf")], [float("-inf"), 1.5, float("inf")]]
stage = Bucketizer().set_input_cols("f1", "f2", "f3", "f4").set_output_cols("o1", "o2", "o3", "o4") \
    .set_splits_array(splits)
out = stage.transform(data)[0]
for row in out.rows():
    print("Input Values: %s \tOutput Values: %s" % (list(row[:4]), list(row[4:])))
