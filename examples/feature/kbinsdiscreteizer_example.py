"""Discretizes continuous features into bins (uniform/quantile/kmeans).

Run: python examples/feature/kbinsdiscreteizer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import KBinsDiscretizer  # noqa: E402
data = Table.from_rows([(Vectors.dense(1, 10, 0),), (Vectors.dense(1, 10, 0),), (Vectors.dense(1, 10, 0),),
                        (Vectors.dense(4, 10, 0),), (Vectors.dense(5, 10, 0),), (Vectors.dense(6, 10, 0),),
                        (Vectors.dense(7, 10, 0),), (Vectors.dense(10, 10, 0),), (Vectors.dense(13, 10, 3),)],
                       ["input"])
model = KBinsDiscretizer().set_num_bins(3).set_strategy("uniform").fit(data)
out = model.transform(data)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
