"""One-hot encodes categorical indices into sparse binary vectors.

Run: python examples/feature/onehotencoder_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import OneHotEncoder  # noqa: E402
train = Table.from_rows([(0.0,), (1.0,), (2.0,), (0.0,)], ["input"])
predict = Table.from_rows([(0.0,), (1.0,), (2.0,)], ["input"])
model = OneHotEncoder().set_input_cols("input").set_output_cols("output").fit(train)
out = model.transform(predict)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
