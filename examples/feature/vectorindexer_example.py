"""Indexes categorical features inside vectors (features with few distinct values).

Run: python examples/feature/vectorindexer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import VectorIndexer  # noqa: E402
train = Table.from_rows([(Vectors.dense(1, 1),), (Vectors.dense(2, -1),), (Vectors.dense(3, 1),),
                         (Vectors.dense(4, 0),), (Vectors.dense(5, 0),)], ["input"])
predict = Table.from_rows([(Vectors.dense(0, 2),), (Vectors.dense(0, 0),), (Vectors.dense(0, -1),)], ["input"])
model = VectorIndexer().set_input_col("input").set_output_col("output").set_handle_invalid("keep") \
    .set_max_categories(3).fit(train)
out = model.transform(predict)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
