"""Normalizes every vector to unit p-norm.

Run: python examples/feature/normalizer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import Normalizer  # noqa: E402
data = Table.from_rows([(Vectors.dense(2.1, 3.1, 1.2, 3.1, 4.6),), (Vectors.dense(1.2, 3.1, 4.6, 2.1, 3.1),)],
                       ["inputVec"])
out = Normalizer().set_input_col("inputVec").set_p(1.5).set_output_col("outputVec").transform(data)[0]
for i, o in zip(out.get_list("inputVec"), out.get_list("outputVec")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
