"""Randomly splits a table into parts by weights.

Run: python examples/feature/randomsplitter_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import RandomSplitter  # noqa: E402
data = Table.from_rows([(i, float(i)) for i in range(10)], ["id", "value"])
parts = RandomSplitter().set_weights(4.0, 6.0).set_seed(0).transform(data)
for k, part in enumerate(parts):
    print("Split %d: %s" % (k, part.get_list("id")))
