"""Runs Pearson's chi-squared independence test.

Run: python examples/stats/chisqtest_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.stats.chisqtest import ChiSqTest  # noqa: E402

data = Table.from_rows([(0., Vectors.dense(5, 1.)), (2., Vectors.dense(6, 2.)), (1., Vectors.dense(7, 2.)),
                        (1., Vectors.dense(5, 4.)), (0., Vectors.dense(5, 1.)), (2., Vectors.dense(6, 2.)),
                        (1., Vectors.dense(7, 2.)), (1., Vectors.dense(5, 4.)), (2., Vectors.dense(5, 1.)),
                        (0., Vectors.dense(5, 2.)), (0., Vectors.dense(5, 2.)), (1., Vectors.dense(9, 4.)),
                        (1., Vectors.dense(9, 3.))], ["label", "features"])
out = ChiSqTest().set_flatten(True).transform(data)[0]
for idx, p, dof, stat in out.rows():
    print("Feature Index: %s \tP Value: %s \tDegree of Freedom: %s \tStatistics: %s" % (idx, p, dof, stat))
