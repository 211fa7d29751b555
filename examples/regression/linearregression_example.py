"""Trains a LinearRegression model and uses it for regression.

Run: python examples/regression/linearregression_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.regression.linearregression import LinearRegression  # noqa: E402

train = Table.from_rows([(Vectors.dense(2, 1), 4., 1.), (Vectors.dense(3, 2), 7., 1.), (Vectors.dense(4, 3), 10., 1.),
                         (Vectors.dense(2, 4), 10., 1.), (Vectors.dense(2, 2), 6., 1.), (Vectors.dense(4, 3), 10., 1.),
                         (Vectors.dense(1, 2), 5., 1.), (Vectors.dense(5, 3), 11., 1.)],
                        ["features", "label", "weight"])
model = LinearRegression().set_weight_col("weight").fit(train)
out = model.transform(train)[0]
for f, label, pred in zip(out.get_list("features"), out.get_list("label"), out.get_list("prediction")):
    print("Features: %s \tExpected Result: %s \tPrediction Result: %s" % (f, label, pred))
