"""Trains an OnlineKMeans model on a stream of mini-batches.

Run: python examples/clustering/onlinekmeans_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.clustering.kmeans import OnlineKMeans  # noqa: E402
from flink_ml_amd.stream import InMemorySource  # noqa: E402

rows = [(Vectors.dense(0.0, 0.0),), (Vectors.dense(0.0, 0.3),), (Vectors.dense(0.3, 0.0),),
              (Vectors.dense(9.0, 0.0),), (Vectors.dense(9.0, 0.6),), (Vectors.dense(9.6, 0.0),)]
init = Table({"centroids": [[Vectors.dense(0.0, 0.0), Vectors.dense(9.0, 9.0)]],
              "weights": [Vectors.dense(0.0, 0.0)]}, num_rows=1)
okm = OnlineKMeans().set_k(2).set_global_batch_size(6).set_decay_factor(0.5).set_initial_model_data(init)
src = InMemorySource()
model = okm.fit(src)
src.add_rows(rows, ["features"])  # one global batch of 6 points -> one model update
src.close()
out = model.transform(Table.from_rows([(Vectors.dense(0.1, 0.1),), (Vectors.dense(9.1, 0.2),)], ["features"]))[0]
for f, c in zip(out.get_list("features"), out.get_list("prediction")):
    print("Features: %s \tCluster ID: %s" % (f, c))
