"""Replaces missing values (NaN) with the column mean/median/most frequent value.

Run: python examples/feature/imputer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import Imputer  # noqa: E402
nan = float("nan")
data = Table.from_rows([(nan, 9.0), (1.0, 9.0), (1.5, 9.0), (2.5, nan), (5.0, 5.0), (5.0, 4.0)], ["input1", "input2"])
model = Imputer().set_input_cols("input1", "input2").set_output_cols("output1", "output2") \
    .set_strategy("mean").set_missing_value(nan).fit(data)
out = model.transform(data)[0]
for i1, i2, o1, o2 in out.select("input1", "input2", "output1", "output2").rows():
    print("Input Values: %s \tOutput Values: %s" % ([i1, i2], [o1, o2]))
