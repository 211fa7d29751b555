"""Removes features whose variance is at most a threshold.

Run: python examples/feature/variancethresholdselector_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import VarianceThresholdSelector  # noqa: E402
data = Table.from_rows([(1, Vectors.dense(5.0, 7.0, 0.0, 7.0, 6.0, 0.0)),
                        (2, Vectors.dense(0.0, 9.0, 6.0, 0.0, 5.0, 9.0)),
                        (3, Vectors.dense(0.0, 9.0, 3.0, 0.0, 5.0, 5.0)),
                        (4, Vectors.dense(1.0, 9.0, 8.0, 5.0, 7.0, 4.0)),
                        (5, Vectors.dense(9.0, 8.0, 6.0, 5.0, 4.0, 4.0)),
                        (6, Vectors.dense(6.0, 9.0, 7.0, 0.0, 2.0, 0.0))], ["id", "input"])
model = VarianceThresholdSelector().set_input_col("input").set_variance_threshold(8.0).fit(data)
out = model.transform(data)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
