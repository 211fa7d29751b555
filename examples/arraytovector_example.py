"""Converts numeric arrays into dense vectors.

Run: python examples/arraytovector_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.functions import array_to_vector  # noqa: E402

arrays = [[0.0, 0.0], [0.0, 1.0], [1.0, 0.0]]
for a, v in zip(arrays, array_to_vector(arrays).tolist()):
    print("Input array: %s \tOutput vector: %s" % (a, Vectors.dense(*v)))
