"""Concatenates numeric and vector columns into one vector column.

Run: python examples/feature/vectorassembler_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import VectorAssembler  # noqa: E402
data = Table.from_rows([(Vectors.dense(2.1, 3.1), 1.0, Vectors.sparse(5, [3], [1.0])),
                        (Vectors.dense(2.1, 3.1), 1.0, Vectors.sparse(5, [4, 2, 3, 1], [4.0, 2.0, 3.0, 1.0]))],
                       ["vec", "num", "sparse_vec"])
stage = VectorAssembler().set_input_cols("vec", "num", "sparse_vec").set_output_col("assembled_vec") \
    .set_input_sizes(2, 1, 5)
out = stage.transform(data)[0]
for vals, o in zip(zip(out.get_list("vec"), out.get_list("num"), out.get_list("sparse_vec")), out.get_list("assembled_vec")):
    print("Input Values: %s \tOutput Value: %s" % (list(vals), o))
