"""Lower-cases text and splits it on whitespace.

Run: python examples/feature/tokenizer_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import Tokenizer  # noqa: E402
data = Table.from_rows([("Test for tokenization.",), ("Te,st. punct",)], ["input"])
out = Tokenizer().set_input_col("input").set_output_col("output").transform(data)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
