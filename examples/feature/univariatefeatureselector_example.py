"""Selects features by univariate statistical tests against the label.

Run: python examples/feature/univariatefeatureselector_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import UnivariateFeatureSelector  # noqa: E402
data = Table.from_rows([(Vectors.dense(1.7, 4.4, 7.6, 5.8, 9.6, 2.3), 3.0),
                        (Vectors.dense(8.8, 7.3, 5.7, 7.3, 2.2, 4.1), 2.0),
                        (Vectors.dense(1.2, 9.5, 2.5, 3.1, 8.7, 2.5), 1.0),
                        (Vectors.dense(3.7, 9.2, 6.1, 4.1, 7.5, 3.8), 2.0),
                        (Vectors.dense(8.9, 5.2, 7.8, 8.3, 5.2, 3.0), 4.0),
                        (Vectors.dense(7.9, 8.5, 9.2, 4.0, 9.4, 2.1), 4.0)], ["features", "label"])
model = UnivariateFeatureSelector().set_features_col("features").set_label_col("label") \
    .set_feature_type("continuous").set_label_type("categorical").set_selection_threshold(1).fit(data)
out = model.transform(data)[0]
for i, o in zip(out.get_list("features"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
