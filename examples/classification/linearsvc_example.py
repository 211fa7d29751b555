"""Trains a LinearSVC model and uses it for classification.

Run: python examples/classification/linearsvc_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.classification.linearsvc import LinearSVC  # noqa: E402

train = Table.from_rows([(Vectors.dense(1, 2, 3, 4), 0., 1.), (Vectors.dense(2, 2, 3, 4), 0., 2.),
                         (Vectors.dense(3, 2, 3, 4), 0., 3.), (Vectors.dense(4, 2, 3, 4), 0., 4.),
                         (Vectors.dense(5, 2, 3, 4), 0., 5.), (Vectors.dense(11, 2, 3, 4), 1., 1.),
                         (Vectors.dense(12, 2, 3, 4), 1., 2.), (Vectors.dense(13, 2, 3, 4), 1., 3.),
                         (Vectors.dense(14, 2, 3, 4), 1., 4.), (Vectors.dense(15, 2, 3, 4), 1., 5.)],
                        ["features", "label", "weight"])
model = LinearSVC().set_weight_col("weight").fit(train)
out = model.transform(train)[0]
for f, label, pred, raw in zip(out.get_list("features"), out.get_list("label"), out.get_list("prediction"),
                               out.get_list("rawPrediction")):
    print("Features: %s \tExpected Result: %s \tPrediction Result: %s \tRaw Prediction Result: %s"
          % (f, label, pred, raw))
