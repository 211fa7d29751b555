"""Selects a subset of vector elements by index.

Run: python examples/feature/vectorslicer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import VectorSlicer  # noqa: E402
data = Table.from_rows([(1, Vectors.dense(2.1, 3.1, 1.2, 3.1, 4.6)), (2, Vectors.dense(1.2, 3.1, 4.6, 2.1, 3.1))],
                       ["id", "vec"])
out = VectorSlicer().set_input_col("vec").set_indices(1, 2, 3).set_output_col("slicedVec").transform(data)[0]
for i, o in zip(out.get_list("vec"), out.get_list("slicedVec")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
