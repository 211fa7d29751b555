"""Trains a Knn model and uses it for classification.

Run: python examples/classification/knn_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.classification.knn import KNN  # noqa: E402

train = Table.from_rows([(Vectors.dense(2.0, 3.0), 1.0), (Vectors.dense(2.1, 3.1), 1.0),
                         (Vectors.dense(200.1, 300.1), 2.0), (Vectors.dense(200.2, 300.2), 2.0),
                         (Vectors.dense(200.3, 300.3), 2.0), (Vectors.dense(200.4, 300.4), 2.0),
                         (Vectors.dense(200.4, 300.4), 2.0), (Vectors.dense(200.6, 300.6), 2.0),
                         (Vectors.dense(2.1, 3.1), 1.0), (Vectors.dense(2.1, 3.1), 1.0),
                         (Vectors.dense(2.1, 3.1), 1.0), (Vectors.dense(2.1, 3.1), 1.0),
                         (Vectors.dense(2.3, 3.2), 1.0), (Vectors.dense(2.3, 3.2), 1.0),
                         (Vectors.dense(2.8, 3.2), 3.0), (Vectors.dense(300., 3.2), 4.0),
                         (Vectors.dense(2.2, 3.2), 1.0), (Vectors.dense(2.4, 3.2), 5.0),
                         (Vectors.dense(2.5, 3.2), 5.0), (Vectors.dense(2.5, 3.2), 5.0),
                         (Vectors.dense(2.1, 3.1), 1.0)], ["features", "label"])
predict = Table.from_rows([(Vectors.dense(4.0, 4.1), 5.0), (Vectors.dense(300, 42), 2.0)], ["features", "label"])
model = KNN().set_k(4).fit(train)
out = model.transform(predict)[0]
for f, label, pred in zip(out.get_list("features"), out.get_list("label"), out.get_list("prediction")):
    print("Features: %s \tExpected Result: %s \tPrediction Result: %s" % (f, label, pred))
