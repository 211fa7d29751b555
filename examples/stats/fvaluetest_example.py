"""Runs the F-value test between continuous features and a continuous label.

Run: python examples/stats/fvaluetest_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.stats.fvaluetest import FValueTest  # noqa: E402

data = Table.from_rows([(0.52516321, Vectors.dense(0.19151945, 0.62210877, 0.43772774, 0.78535858, 0.77997581)),
                        (0.88275782, Vectors.dense(0.27259261, 0.27646426, 0.80187218, 0.95813935, 0.87593263)),
                        (0.67524507, Vectors.dense(0.35781727, 0.50099513, 0.68346294, 0.71270203, 0.37025075)),
                        (0.76734274, Vectors.dense(0.56119619, 0.50308317, 0.01376845, 0.77282662, 0.88264119)),
                        (0.73909146, Vectors.dense(0.36488598, 0.61539618, 0.07538124, 0.36882401, 0.9331401)),
                        (0.83628749, Vectors.dense(0.65137814, 0.39720258, 0.78873014, 0.31683612, 0.56809865))],
                       ["label", "features"])
out = FValueTest().set_flatten(True).transform(data)[0]
for idx, p, dof, f in out.rows():
    print("Feature Index: %s \tP Value: %s \tDegree of Freedom: %s \tF Value: %s" % (idx, p, dof, f))
