"""Standardizes features to zero mean and/or unit variance.

Run: python examples/feature/standardscaler_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import StandardScaler  # noqa: E402
data = Table.from_rows([(Vectors.dense(-2.5, 9, 1),), (Vectors.dense(1.4, -5, 1),), (Vectors.dense(2, -1, -2),)],
                       ["input"])
model = StandardScaler().fit(data)
out = model.transform(data)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
