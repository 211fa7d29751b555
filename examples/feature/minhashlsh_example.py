"""MinHash LSH: hashing, approximate nearest neighbours and similarity join.

Run: python examples/feature/minhashlsh_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import MinHashLSH  # noqa: E402
dataA = Table.from_rows([(0, Vectors.sparse(6, [0, 1, 2], [1.0, 1.0, 1.0])),
                         (1, Vectors.sparse(6, [2, 3, 4], [1.0, 1.0, 1.0])),
                         (2, Vectors.sparse(6, [0, 2, 4], [1.0, 1.0, 1.0]))], ["id", "vec"])
dataB = Table.from_rows([(3, Vectors.sparse(6, [1, 3, 5], [1.0, 1.0, 1.0])),
                         (4, Vectors.sparse(6, [2, 3, 5], [1.0, 1.0, 1.0])),
                         (5, Vectors.sparse(6, [1, 2, 4], [1.0, 1.0, 1.0]))], ["id", "vec"])
model = MinHashLSH().set_input_col("vec").set_output_col("hashes").set_seed(2022) \
    .set_num_hash_tables(5).set_num_hash_functions_per_table(3).fit(dataA)
out = model.transform(dataA)[0]
for i, h in zip(out.get_list("id"), out.get_list("hashes")):
    print("id: %s \tHash values: %s" % (i, h))
key = Vectors.dense(1.0, 1.0, 1.0, 0.0, 0.0, 0.0)
nn = model.approx_nearest_neighbors(dataA, key, 2)
for i, d in zip(nn.get_list("id"), nn.get_list("distCol")):
    print("Nearest neighbour id: %s \tdistance: %s" % (i, d))
join = model.approx_similarity_join(dataA, dataB, 0.6, "id")
for row in join.rows():
    print("Similarity join (idA, idB, distance): %s" % (row,))
