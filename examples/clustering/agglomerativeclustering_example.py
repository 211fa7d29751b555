"""Clusters points hierarchically with AgglomerativeClustering.

Run: python examples/clustering/agglomerativeclustering_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.clustering.agglomerativeclustering import AgglomerativeClustering  # noqa: E402

data = Table.from_rows([(Vectors.dense(1, 1),), (Vectors.dense(1, 4),), (Vectors.dense(1, 0),),
                        (Vectors.dense(4, 1.5),), (Vectors.dense(4, 4),), (Vectors.dense(4, 0),)], ["features"])
ac = AgglomerativeClustering().set_linkage("ward").set_distance_measure("euclidean").set_prediction_col("prediction")
out, merges = ac.transform(data)
for f, c in zip(out.get_list("features"), out.get_list("prediction")):
    print("Features: %s \tCluster ID: %s" % (f, c))
for row in merges.rows():
    print("Merge: clusterId1=%s clusterId2=%s distance=%s size=%s" % row)
