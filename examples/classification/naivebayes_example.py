"""Trains a NaiveBayes model and uses it for classification.

Run: python examples/classification/naivebayes_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.classification.naivebayes import NaiveBayes  # noqa: E402

train = Table.from_rows([(Vectors.dense(0, 0.), 11.), (Vectors.dense(1, 0), 10.), (Vectors.dense(1, 1.), 10.)],
                        ["features", "label"])
predict = Table.from_rows([(Vectors.dense(0, 1.),), (Vectors.dense(0, 0.),), (Vectors.dense(1, 0),),
                           (Vectors.dense(1, 1.),)], ["features"])
model = NaiveBayes().set_smoothing(1.0).fit(train)
out = model.transform(predict)[0]
for f, pred in zip(out.get_list("features"), out.get_list("prediction")):
    print("Features: %s \tPrediction Result: %s" % (f, pred))
