"""Computes the interaction (outer product) of numeric and vector columns.

Run: python examples/feature/interaction_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import Interaction  # noqa: E402
data = Table.from_rows([(1, Vectors.dense(1, 2), Vectors.dense(3, 4)), (2, Vectors.dense(2, 8), Vectors.dense(3, 4))],
                       ["f0", "f1", "f2"])
out = Interaction().set_input_cols("f0", "f1", "f2").set_output_col("interaction_vec").transform(data)[0]
for vals, o in zip(zip(out.get_list("f0"), out.get_list("f1"), out.get_list("f2")), out.get_list("interaction_vec")):
    print("Input Values: %s \tOutput Value: %s" % (list(vals), o))
