"""Maps string (or numeric) columns to indices ordered by frequency or alphabet.

Run: python examples/feature/stringindexer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import StringIndexer  # noqa: E402
train = Table.from_rows([("a", 1.0), ("b", 1.0), ("b", 2.0), ("c", 0.0), ("d", 2.0), ("a", 2.0), ("b", 2.0),
                         ("b", -1.0), ("a", -1.0), ("c", -1.0)], ["inputCol1", "inputCol2"])
predict = Table.from_rows([("a", 2.0), ("b", 1.0), ("c", 2.0)], ["inputCol1", "inputCol2"])
model = StringIndexer().set_string_order_type("alphabetAsc").set_input_cols("inputCol1", "inputCol2") \
    .set_output_cols("outputCol1", "outputCol2").fit(train)
out = model.transform(predict)[0]
for row in out.rows():
    print("Input Values: %s \tOutput Values: %s" % (list(row[:2]), list(row[2:])))
