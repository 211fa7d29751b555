"""Converts a vector column into double arrays.

Run: python examples/vectortoarray_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.functions import vector_to_array  # noqa: E402

t = Table.from_rows([(1, Vectors.dense(1.0, 2.0, 3.0)), (2, Vectors.sparse(3, [1], [4.0]))], ["id", "vec"])
for vec, arr in zip(t.get_list("vec"), vector_to_array(t, "vec")):
    print("Input vector: %s \tOutput array: %s" % (vec, [float(x) for x in arr]))
