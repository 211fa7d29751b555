"""Applies the orthonormal DCT-II to dense vectors.

Run: python examples/feature/dct_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import DCT  # noqa: E402
data = Table.from_rows([(Vectors.dense(1.0, 1.0, 1.0, 1.0),), (Vectors.dense(1.0, 0.0, -1.0, 0.0),)], ["input"])
out = DCT().transform(data)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
