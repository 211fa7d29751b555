"""Scales features using statistics robust to outliers (median and IQR).

Run: python examples/feature/robustscaler_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import RobustScaler  # noqa: E402
train = Table.from_rows([(i, Vectors.dense(float(i), -float(i))) for i in range(10)], ["id", "input"])
predict = Table.from_rows([(Vectors.dense(3.0, -3.0),), (Vectors.dense(6.0, -6.0),), (Vectors.dense(99.0, -99.0),)],
                          ["input"])
model = RobustScaler().set_input_col("input").set_output_col("output").set_lower(0.25).set_upper(0.75) \
    .set_relative_error(0.001).set_with_centering(True).set_with_scaling(True).fit(train)
out = model.transform(predict)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
