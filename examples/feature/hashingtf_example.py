"""Maps token sequences to term-frequency vectors via the hashing trick.

Run: python examples/feature/hashingtf_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402,F401
from flink_ml_amd.lib.feature import HashingTF  # noqa: E402
data = Table.from_rows([(["HashingTFTest", "Hashing", "Term", "Frequency", "Test"],),
                        (["HashingTFTest", "Hashing", "Hashing", "Test", "Test"],)], ["input"])
out = HashingTF().set_input_col("input").set_output_col("output").set_num_features(128).transform(data)[0]
for i, o in zip(out.get_list("input"), out.get_list("output")):
    print("Input Value: %s \tOutput Value: %s" % (i, o))
