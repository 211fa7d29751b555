"""Trains an OnlineLogisticRegression model on a stream and predicts with the latest model.

Run: python examples/classification/onlinelogisticregression_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.classification.logisticregression import OnlineLogisticRegression  # noqa: E402
from flink_ml_amd.stream import InMemorySource  # noqa: E402

train_rows = [(Vectors.dense(0.1, 2.), 0.), (Vectors.dense(0.2, 2.), 0.), (Vectors.dense(0.3, 2.), 0.),
              (Vectors.dense(0.4, 2.), 0.), (Vectors.dense(0.5, 2.), 0.), (Vectors.dense(11., 12.), 1.),
              (Vectors.dense(12., 11.), 1.), (Vectors.dense(13., 12.), 1.), (Vectors.dense(14., 12.), 1.),
              (Vectors.dense(15., 12.), 1.)]
src = InMemorySource()
init = Table.from_rows([(Vectors.dense(0.41233679404769874, -0.18088118293232122), 0)], ["coefficient", "modelVersion"])
olr = OnlineLogisticRegression().set_features_col("features").set_label_col("label").set_global_batch_size(10) \
    .set_initial_model_data(init)
model = olr.fit(src)
src.add_rows(train_rows, ["features", "label"])  # one global batch -> model version 1
src.close()
predict = Table.from_rows([(Vectors.dense(100, -100),), (Vectors.dense(-100, 100),)], ["features"])
out = model.transform(predict)[0]
for f, pred, raw, ver in zip(out.get_list("features"), out.get_list("prediction"), out.get_list("rawPrediction"),
                             out.get_list("modelVersion")):
    print("Features: %s \tPrediction: %s \tRaw Prediction: %s \tModel Version: %s" % (f, pred, raw, ver))
