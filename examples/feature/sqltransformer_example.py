"""Applies a SQL statement to a table.

Run: python examples/feature/sqltransformer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import SQLTransformer  # noqa: E402
data = Table.from_rows([(0, 1.0, 3.0), (2, 2.0, 5.0)], ["id", "v1", "v2"])
stage = SQLTransformer().set_statement("SELECT *, (v1 + v2) AS v3, (v1 * v2) AS v4 FROM __THIS__")
out = stage.transform(data)[0]
print(out.column_names)
for row in out.rows():
    print(row)
