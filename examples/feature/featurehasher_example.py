"""Hashes numeric, boolean and string columns into one sparse feature vector.

Run: python examples/feature/featurehasher_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import FeatureHasher  # noqa: E402
data = Table.from_rows([(0, "a", 1.0, True), (1, "c", 1.0, False)], ["id", "f0", "f1", "f2"])
stage = FeatureHasher().set_input_cols("f0", "f1", "f2").set_categorical_cols("f0", "f2") \
    .set_output_col("vec").set_num_features(1000)
out = stage.transform(data)[0]
for vals, o in zip(zip(out.get_list("f0"), out.get_list("f1"), out.get_list("f2")), out.get_list("vec")):
    print("Input Values: %s \tOutput Value: %s" % (list(vals), o))
