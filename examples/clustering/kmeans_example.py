"""Trains a KMeans model and uses it for clustering.

Run: python examples/clustering/kmeans_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.clustering.kmeans import KMeans  # noqa: E402

data = Table.from_rows([(Vectors.dense(0.0, 0.0),), (Vectors.dense(0.0, 0.3),), (Vectors.dense(0.3, 3.0),),
                        (Vectors.dense(9.0, 0.0),), (Vectors.dense(9.0, 0.6),), (Vectors.dense(9.6, 0.0),)],
                       ["features"])
model = KMeans().set_k(2).set_seed(1).fit(data)
out = model.transform(data)[0]
for f, c in zip(out.get_list("features"), out.get_list("prediction")):
    print("Features: %s \tCluster ID: %s" % (f, c))
