"""Runs the ANOVA F-test between continuous features and a categorical label.

Run: python examples/stats/anovatest_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.stats.anovatest import ANOVATest  # noqa: E402

data = Table.from_rows([(3, Vectors.dense(0.85956061, 0.1645695, 0.48347596, 0.92102727, 0.42855644, 0.05746009)),
                        (2, Vectors.dense(0.92500743, 0.65760154, 0.13295284, 0.53344893, 0.8994776, 0.24836496)),
                        (1, Vectors.dense(0.03017182, 0.07244715, 0.87416449, 0.55843035, 0.91604736, 0.63346045)),
                        (5, Vectors.dense(0.28325261, 0.36536881, 0.09223386, 0.37251258, 0.34742278, 0.70517077)),
                        (4, Vectors.dense(0.64850904, 0.04090877, 0.21173176, 0.00148992, 0.13897166, 0.21182539)),
                        (4, Vectors.dense(0.02609493, 0.44608735, 0.44910669, 0.35604431, 0.83602659, 0.68693982)),
                        (1, Vectors.dense(0.57766122, 0.90223209, 0.2211755, 0.53287691, 0.2849074, 0.51652598)),
                        (1, Vectors.dense(0.62357837, 0.73111581, 0.86463844, 0.10014373, 0.56908648, 0.20307072))],
                       ["label", "features"])
out = ANOVATest().set_flatten(True).transform(data)[0]
for idx, p, dof, f in out.rows():
    print("Feature Index: %s \tP Value: %s \tDegree of Freedom: %s \tF Value: %s" % (idx, p, dof, f))
