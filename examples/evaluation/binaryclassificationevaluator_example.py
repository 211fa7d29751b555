"""Computes AUC and other binary-classification metrics.

Run: python examples/evaluation/binaryclassificationevaluator_example.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

from flink_ml_amd import Table, Vectors  # noqa: E402
from flink_ml_amd.lib.evaluation.binaryclassificationevaluator import BinaryClassificationEvaluator  # noqa: E402

data = Table.from_rows([(1.0, Vectors.dense(0.1, 0.9)), (1.0, Vectors.dense(0.2, 0.8)),
                        (1.0, Vectors.dense(0.3, 0.7)), (0.0, Vectors.dense(0.25, 0.75)),
                        (0.0, Vectors.dense(0.4, 0.6)), (1.0, Vectors.dense(0.35, 0.65)),
                        (1.0, Vectors.dense(0.45, 0.55)), (0.0, Vectors.dense(0.6, 0.4)),
                        (0.0, Vectors.dense(0.7, 0.3)), (1.0, Vectors.dense(0.65, 0.35)),
                        (0.0, Vectors.dense(0.8, 0.2)), (1.0, Vectors.dense(0.9, 0.1))], ["label", "rawPrediction"])
ev = BinaryClassificationEvaluator().set_metrics_names("areaUnderPR", "ks", "areaUnderROC")
out = ev.transform(data)[0]
row = out.rows()[0]
print("Area under the precision-recall curve: %s" % row[0])
print("Kolmogorov-Smirnov value: %s" % row[1])
print("Area under the receiver operating characteristic curve: %s" % row[2])
