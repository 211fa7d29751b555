"""Scales every feature into [-1, 1] by its maximum absolute value.

Run: python examples/feature/maxabsscaler_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import MaxAbsScaler  # noqa: E402
train = Table.from_rows([(Vectors.dense(0.0, 3.0),), (Vectors.dense(2.1, 0.0),), (Vectors.dense(4.1, 5.1),),
                         (Vectors.dense(6.1, 8.1),), (Vectors.dense(200, 400),)], ["input"])
predict = Table.from_rows([(Vectors.dense(150.0, 90.0),), (Vectors.dense(50.0, 40.0),),
                           (Vectors.dense(100.0, 50.0),)], ["input"])
model = MaxAbsScaler().fit(train)
out = model.transform(predict)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
