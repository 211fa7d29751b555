"""Maps indices back to the strings of a StringIndexer-style model.

Run: python examples/feature/indextostringmodel_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import IndexToStringModel  # noqa: E402
model_data = Table.from_rows([([["a", "b", "c", "d"], ["-1.0", "0.0", "1.0", "2.0"]],)], ["stringArrays"])
data = Table.from_rows([(0, 3), (1, 2)], ["inputCol1", "inputCol2"])
model = IndexToStringModel().set_input_cols("inputCol1", "inputCol2") \
    .set_output_cols("outputCol1", "outputCol2").set_model_data(model_data)
out = model.transform(data)[0]
for row in out.rows():
    print("Input Values: %s \tOutput Values: %s" % (list(row[:2]), list(row[2:])))
